"""Does torch's fp32 GEMM write every element of an output larger than 2 GiB?

The reference scores of the 2M-row index tests ([256, 2097485] fp32 = 2^31 + 340992 bytes) came
back with garbage only in the elements past byte 2^31, and only after other tests had dirtied
the allocator's memory.  This fills the output with a sentinel first, then compares against a
row-chunked product.
"""
import torch

torch.manual_seed(0)
dev = "cuda"
for n in ((1 << 21) - 4096, (1 << 21) + 333):
    a = torch.randn(256, 384, device=dev)
    b = torch.randn(n, 384, device=dev)
    out = torch.full((256, n), float("nan"), device=dev)
    torch.mm(a, b.t(), out=out)
    ref = torch.cat([a @ b[s:s + (1 << 19)].t() for s in range(0, n, 1 << 19)], 1)
    bad = ~torch.isclose(out, ref, atol=1e-3, rtol=1e-4)
    nb = int(bad.sum())
    first = int(bad.flatten().nonzero()[0]) * 4 if nb else -1
    print(f"n={n} bytes={256 * n * 4} (2^31 = {1 << 31}) wrong={nb} first_wrong_byte={first}",
          flush=True)
    del a, b, out, ref, bad
    torch.cuda.empty_cache()
