"""CU-partitioned streams (include/mam_stream.h): the mask split is host-only arithmetic, checked here without a GPU."""
import numpy as np
import pytest

from mam3slam_amd import streams
from mam3slam_amd._lib import MamError


def _bits(m, n):
    return np.array([(int(m[i >> 5]) >> (i & 31)) & 1 for i in range(n)], bool)


@pytest.mark.parametrize("eighths", [2, 4, 6])
def test_cu_mask_split_partitions_every_xcd(eighths):
    n = 256
    a, b = _bits(streams.cu_mask(n, eighths), n), _bits(streams.cu_mask(n, eighths, complement=True), n)
    assert not (a & b).any() and (a | b).all()
    assert a.sum() == n * eighths // 8
    # the same share of every XCD's CUs whether the mask bits map to XCDs as contiguous 32-bit runs or interleaved
    for x in range(8):
        assert a[32 * x:32 * x + 32].sum() == 32 * eighths // 8
        assert a[x::8].sum() == 32 * eighths // 8


@pytest.mark.parametrize("eighths", [0, 1, 3, 8])
def test_cu_mask_split_rejects_uneven_shares(eighths):
    with pytest.raises(MamError):
        streams.cu_mask(256, eighths)
