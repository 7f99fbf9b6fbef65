"""Import shim: the package directory is ``covid-spings-variant-caller_amd/`` (hyphenated, per the
repo layout), which Python cannot import by name.  ``import spings`` registers it as the module
``covid_spings_variant_caller_amd`` and returns it."""
import importlib.util
import os
import sys

_NAME = "covid_spings_variant_caller_amd"
_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "covid-spings-variant-caller_amd")


def _load():
    if _NAME in sys.modules:
        return sys.modules[_NAME]
    spec = importlib.util.spec_from_file_location(_NAME, os.path.join(_DIR, "__init__.py"),
                                                  submodule_search_locations=[_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[_NAME] = mod
    spec.loader.exec_module(mod)
    return mod


pkg = _load()
