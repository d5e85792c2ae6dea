"""Host cost of the MiniLM encoder forward per call: eager launches vs hipGraph replay (host time
of the call alone, no sync inside the timed loop; the GPU runs behind).

    python benchmarks/diag/graph_host.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch

    cfg = get_config("minilm-l6")
    enc = HipEncoder(cfg, seed=0, device="cuda")
    b = synthetic_batch(cfg, 256, 128, seed=0).to("cuda")
    o32 = torch.empty(256, cfg.hidden, device="cuda")
    ou = torch.empty(256, cfg.hidden, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        enc.forward_packed(b, o32, ou)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        enc.forward_packed(b, o32, ou)
    torch.cuda.synchronize()
    out = {}
    for name, f in (("eager", lambda: enc.forward_packed(b, o32, ou)), ("graph", g.replay)):
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        n = 50
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[name] = {"host_ms_per_call": round((t1 - t0) * 1e3 / n, 3),
                     "wall_ms_per_call": round((t2 - t0) * 1e3 / n, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
