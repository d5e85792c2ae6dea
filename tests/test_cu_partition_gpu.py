"""CU-masked streams on the GPU: the runtime reports the masks CuPartition asked for (scan stream
= every CU but the balanced reserve, side streams = every CU or the reserve) and work on the
masked streams computes correctly, in order with the default stream through events."""
import pytest
import torch

from codename_symbiont_amd.parallel.cu_partition import CuPartition, mask_words

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("side_all", [True, False])
def test_cu_partition_masks_and_work(side_all):
    p = CuPartition("cuda", 2, side_all=side_all, n_side=2)
    assert p.n_cus == 256 and p.main_cus == 256 - 16 and len(p.reserve) == 16
    main, side = p.masks()
    assert main == mask_words(p.n_cus, [c for c in range(p.n_cus) if c not in p.reserve])
    assert side == (mask_words(p.n_cus, range(p.n_cus)) if side_all else mask_words(p.n_cus, p.reserve))
    x = torch.randn(1 << 20, device="cuda")
    ev = torch.cuda.Event()
    ev.record()
    outs = []
    for st in (p.main, *p.sides):
        st.wait_event(ev)
        with torch.cuda.stream(st):
            outs.append((x * 2 + 1).sum())
    for st in (p.main, *p.sides):
        torch.cuda.current_stream().wait_stream(st)
    want = (x * 2 + 1).sum()
    for o in outs:
        torch.testing.assert_close(o, want)


def test_cu_probe_reads_hardware_ids():
    """probe_cu_map: every probed mask bit's launch reports valid hardware ids (XCC 0..7); the
    workgroups of one single-bit launch are NOT confined to one CU on this driver (the reason the
    partition uses balanced_reserve), which the probe reports as a set per bit."""
    from codename_symbiont_amd.parallel.cu_partition import probe_cu_map

    m = probe_cu_map("cuda", bits=[0, 1, 37, 255])
    assert len(m) == 4
    for ids in m:
        assert ids and all(0 <= x < 8 and 0 <= se < 8 and 0 <= cu < 16 for x, se, cu in ids)
