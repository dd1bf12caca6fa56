"""LzmaBench harness restatement (lzma_amd/lzmabench.py vs LzmaBench.java:226-403).

CPU: the rating arithmetic and the printed format, checked against values
worked by hand from the Java formulas. GPU: one pass at the smallest allowed
dictionary, whose output lines must parse and whose CRC checks must pass.
"""
import io
import re

import pytest

from lzma_amd import lzmabench as lb


def test_get_log_size_matches_java_table():
    # LzmaBench.java:228-237: exact powers of two give (i << 8), the steps between
    # them are 1/256 of the power
    assert lb.get_log_size(1 << 18) == 18 << 8
    assert lb.get_log_size(1 << 21) == 21 << 8
    assert lb.get_log_size((1 << 21) + 1) == (21 << 8) + 1
    assert lb.get_log_size((1 << 21) + (1 << 13)) == (21 << 8) + 1
    assert lb.get_log_size((1 << 21) + (1 << 13) + 1) == (21 << 8) + 2
    assert lb.get_log_size(1) == 8 << 8


def test_ratings_match_java_formulas():
    # dict 2^21: t = 3 << 8 = 768; 1060 + (768 * 768 * 10 >> 16) = 1060 + 90 = 1150 commands per byte
    assert lb.get_compress_rating(1 << 21, 1000, 1 << 20) == (1 << 20) * 1150
    assert lb.get_compress_rating(1 << 18, 2000, 1000) == 1000 * 1060 * 1000 // 2000
    assert lb.get_decompress_rating(500, 4096, 1024) == (1024 * 220 + 4096 * 20) * 1000 // 500
    assert lb.my_mult_div64(12345, 0) == 12345 * 1000   # elapsed 0 -> 1 ms (LzmaBench.java:246-248)


def test_results_line_format():
    line = lb.results(1 << 21, 1000, 3 << 20, False, 0)
    # PrintValue right-aligns in 6 columns, then " KB/s  ", the rating in MIPS
    assert line == "  3072 KB/s    3617 MIPS"
    dline = lb.results(1 << 21, 100, 3 << 20, True, 1 << 20)
    assert re.fullmatch(r" {0,5}\d+ KB/s  {1,6}\d+ MIPS", dline)


def test_small_dictionary_rejected_like_java():
    out = io.StringIO()
    assert lb.lzma_benchmark(1, 1 << 17, out=out) == 1
    assert "must be >= 18" in out.getvalue()


@pytest.mark.gpu
def test_lzmabench_one_pass_on_gpu():
    out = io.StringIO()
    assert lb.lzma_benchmark(1, 1 << 18, out=out, copies=4) == 0
    lines = out.getvalue().strip().splitlines()
    assert lines[0].strip().startswith("Compressing")
    assert lines[-1].endswith("Average")
    assert len(re.findall(r"KB/s", lines[-1])) == 2
