"""CPU: the native Spark-2.1 libsvm reader (fm_read_libsvm) against the oracle's restatement
of MLUtils.parseLibSVMFile, on the reference's own data file (tests/golden/sample.txt) and
on edge cases of the format."""

import os

import numpy as np
import pytest

from oracle.libsvm_ref import parse_libsvm

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _native(path):
    from fm_spark_amd.data import read_libsvm_csr

    return read_libsvm_csr(path)


def _same(a, b):
    for x, y in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, y)
    assert a[4] == b[4]


def test_sample_txt_matches_restatement():
    path = os.path.join(GOLD, "sample.txt")
    got = _native(path)
    _same(got, parse_libsvm(open(path).read()))
    assert len(got[0]) > 0


@pytest.mark.parametrize("text", [
    "1 1:0.5 3:2\n0 2:1e-3\n",
    "# header comment\n\n   2.5   1:1  4:-0.25   \n\n0\n-1 7:3.0\n",      # blanks, padding, empty row
    "1\t\n0 1:1\n",                                                        # trimmed tab
    "3 2:1:9 5:4\n",                                                       # extra ':' field ignored
    "",                                                                    # empty file
    "0\n0\n",                                                              # only empty rows
])
def test_edge_cases(tmp_path, text):
    p = tmp_path / "d.txt"
    p.write_text(text)
    _same(_native(str(p)), parse_libsvm(text))


@pytest.mark.parametrize("text", ["1 3:1 2:1\n", "1 0:1\n", "1 1:x\n", "abc 1:1\n", "1 2\n"])
def test_malformed_lines_raise(tmp_path, text):
    from fm_spark_amd._native import FMError

    p = tmp_path / "bad.txt"
    p.write_text(text)
    with pytest.raises(FMError):
        _native(str(p))
    with pytest.raises((ValueError, IndexError)):  # Java: NumberFormat / ArrayIndexOutOfBounds
        parse_libsvm(text)


def test_missing_file_raises(tmp_path):
    from fm_spark_amd._native import FMError

    with pytest.raises(FMError):
        _native(str(tmp_path / "nope.txt"))
