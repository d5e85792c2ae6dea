#!/usr/bin/env python3
"""Pin the operand layout of v_mfma_scale_f32_32x32x64_f8f6f4 for the fp6 formats (and recheck
fp4 / fp8) on the GPU: random codes packed under a hypothesis, one MFMA (index_stream.hip
mfma_f8f6f4_probe_kernel), compared with the fp32 product of the decoded values.

Hypothesis H1: lane l supplies row / column l & 31, k = 32 (l >> 5) .. + 31; its 32 elements are
packed little-endian, element j at bits [b j, b j + b) of the lane's dwords (b = 8 / 6 / 4).
Prints one JSON line per format: max |error| and whether H1 holds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def e2m3_table():
    v = [m / 8 for m in range(8)]                       # subnormals (exp 0)
    for e in range(1, 4):
        v += [2.0 ** (e - 1) * (1 + m / 8) for m in range(8)]
    return torch.tensor(v + [-x for x in v])            # code c: sign bit 5


def e3m2_table():
    v = [m / 4 * 2.0 ** -2 for m in range(4)]           # subnormals, bias 3
    for e in range(1, 8):
        v += [2.0 ** (e - 3) * (1 + m / 4) for m in range(4)]
    return torch.tensor(v + [-x for x in v])


def e2m1_table():
    v = [0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0]
    return torch.tensor(v + [-x for x in v])


def e4m3_table():
    t = torch.arange(256, dtype=torch.uint8).view(torch.float8_e4m3fn).float()
    return torch.nan_to_num(t, nan=0.0)


def pack(codes, bits):
    """codes [64, 32] ints -> [64, 8] int32 dwords, element j at bits [bits j, bits j + bits)."""
    out = torch.zeros(64, 8, dtype=torch.int64)
    for j in range(32):
        pos = bits * j
        w, o = pos // 32, pos % 32
        c = codes[:, j].long()
        out[:, w] |= (c << o) & 0xFFFFFFFF
        if o + bits > 32:
            out[:, w + 1] |= c >> (32 - o)
    out = torch.where(out >= 2 ** 31, out - 2 ** 32, out)
    return out.to(torch.int32)


def main():
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    h, st = hip(), stream_handle()
    g = torch.Generator().manual_seed(3)
    for fmt, bits, table in ((2, 6, e2m3_table()), (3, 6, e3m2_table()), (4, 4, e2m1_table()),
                             (0, 8, e4m3_table())):
        n_codes = 1 << bits
        ca = torch.randint(0, n_codes, (64, 32), generator=g)
        cb = torch.randint(0, n_codes, (64, 32), generator=g)
        if fmt == 0:   # (skip the NaN codes of e4m3)
            ca[(ca & 0x7F) == 0x7F] = 0
            cb[(cb & 0x7F) == 0x7F] = 0
        va, vb = table[ca], table[cb]
        # A [32 rows, 64 k]: lane l -> row l & 31, k 32 (l >> 5) + j
        A = torch.zeros(32, 64)
        B = torch.zeros(64, 32)
        for l in range(64):
            A[l & 31, 32 * (l >> 5):32 * (l >> 5) + 32] = va[l]
            B[32 * (l >> 5):32 * (l >> 5) + 32, l & 31] = vb[l]
        ref = A @ B
        a = pack(ca, bits).cuda()
        b = pack(cb, bits).cuda()
        sc = torch.full((64,), 127, dtype=torch.int32, device="cuda")
        out = torch.empty(64, 16, device="cuda")
        h.mfma_f8f6f4_probe(a.data_ptr(), b.data_ptr(), sc.data_ptr(), sc.data_ptr(),
                            out.data_ptr(), fmt, st)
        torch.cuda.synchronize()
        got = torch.zeros(32, 32)
        o = out.cpu()
        for l in range(64):
            for r in range(16):
                got[(r & 3) + 8 * (r >> 2) + 4 * (l >> 5), l & 31] = o[l, r]
        err = float((got - ref).abs().max())
        print(json.dumps({"fmt": fmt, "bits": bits, "max_err": err, "ref_absmax": float(ref.abs().max()),
                          "H1": err <= 1e-3 * max(1.0, float(ref.abs().max()))}), flush=True)


if __name__ == "__main__":
    main()
