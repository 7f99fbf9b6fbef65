"""Writes tests/golden/testfile_pileup.npz: the CSR pileup of the reference's own test fixture
(test/testdata/testfile.sam, copied here as testfile.sam) computed by oracle/pileup_port.py with
pysam's pileup() defaults.  Parity unpinned (no pysam/htslib in this image); the fixture freezes
the restatement so both implementations are held to it."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import pileup_port as pp  # noqa: E402

pb, off, codes, quals = pp.to_csr(pp.pileup_columns(os.path.join(HERE, "testfile.sam"), "NC_045512.2"))
np.savez_compressed(os.path.join(HERE, "testfile_pileup.npz"), pos_begin=np.int64(pb), offsets=off, codes=codes,
                    quals=quals)
print(pb, len(off) - 1, len(codes))
