"""parallel/cu_partition.py: the CU reserve is balanced over the 8 XCDs under either CU numbering
(contiguous: XCD = cu // 32, round-robin: XCD = cu % 8) and the stream masks are its exact
complement / the reserve (the GPU test checks the masks the runtime reports)."""
import pytest

from codename_symbiont_amd.parallel.cu_partition import balanced_reserve, mask_words


@pytest.mark.parametrize("per_xcd", [1, 2, 3, 4])
def test_reserve_is_balanced_under_both_numberings(per_xcd):
    r = balanced_reserve(256, per_xcd)
    assert len(r) == 8 * per_xcd and len(set(r)) == len(r)
    for xcd_of in (lambda c: c // 32, lambda c: c % 8):
        counts = [0] * 8
        for c in r:
            counts[xcd_of(c)] += 1
        assert counts == [per_xcd] * 8


def test_mask_words_and_limits():
    assert mask_words(256, [0, 31, 32, 255]) == [0x80000001, 1, 0, 0, 0, 0, 0, 0x80000000]
    assert balanced_reserve(256, 0) == []
    with pytest.raises(ValueError):
        balanced_reserve(256, 5)
    with pytest.raises(ValueError):
        mask_words(64, [64])


def test_reserve_from_a_measured_map_spreads_over_xcc_and_se():
    from codename_symbiont_amd.parallel.cu_partition import reserve_from_map

    # a made-up numbering: bit b -> XCC (b // 4) % 8, SE (b // 32) % 4, CU b % 4 + 4 * (b // 128)
    m = [((b // 4) % 8, (b // 32) % 4, b % 4 + 4 * (b // 128)) for b in range(256)]
    assert len(set(m)) == 256
    r = reserve_from_map(m, 4)
    assert len(r) == 32
    for x in range(8):
        mine = [m[b] for b in r if m[b][0] == x]
        assert len(mine) == 4 and len({se for _, se, _ in mine}) == 4   # one per shader engine
