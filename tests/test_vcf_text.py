"""write_vcf fallback writer: the text pysam.VariantFile writes for the reference's header
(live_variant_caller.py:233-297) — header lines, record sort order, float32 %g fields."""
import numpy as np

import spings  # noqa: F401
from covid_spings_variant_caller_amd.live_variant_caller import write_vcf_text


def test_vcf_text(tmp_path):
    recs = [
        {"start": 240, "stop": 241, "alleles": ("C", "T"), "qual": np.float64(0.00012345678),
         "info": {"DP": 1000, "AD": 990, "GL": 0, "PL": 0, "SCORE": 0}},
        {"start": 3036, "stop": 3037, "alleles": ("c", "A"), "qual": np.float64(1.5e-05),
         "info": {"DP": 25, "AD": 12, "GL": -123.45678901, "PL": 1235, "SCORE": 37}},
    ]
    p = tmp_path / "o.vcf"
    write_vcf_text(str(p), [("NC_045512.2", 29903), ("other", 10)], recs)
    lines = p.read_text().splitlines()
    assert lines[0] == "##fileformat=VCFv4.2"
    assert lines[1] == '##FILTER=<ID=PASS,Description="All filters passed">'
    assert lines[2] == '##INFO=<ID=DP,Number=1,Type=Integer,Description="Total Depth">'
    assert lines[6] == '##INFO=<ID=SCORE,Number=1,Type=Float,Description="Custom scoring function">'
    assert lines[7] == "##contig=<ID=NC_045512.2,length=29903>"
    assert lines[8] == "##contig=<ID=other,length=10>"
    assert lines[9] == "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO"
    assert lines[10] == "NC_045512.2\t241\t.\tC\tT\t0.000123457\t.\tDP=1000;AD=990;GL=0;PL=0;SCORE=0"
    assert lines[11] == "NC_045512.2\t3037\t.\tc\tA\t1.5e-05\t.\tDP=25;AD=12;GL=-123.457;PL=1235;SCORE=37"
    assert len(lines) == 12
