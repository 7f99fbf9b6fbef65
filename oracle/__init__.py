"""ORACLE package — CPU restatements of the reference path, test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it,
and only as the checker.  The product (covid-spings-variant-caller_amd/) never does.
"""
