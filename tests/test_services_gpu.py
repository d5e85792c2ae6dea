"""Service-path tests on the GPU: the micro-batched HIP encoder pipeline and the full
ingest -> HBM index -> semantic search flow with the HIP kernels doing the work."""
import asyncio

import httpx
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_embed_batcher_pipeline_matches_oracle():
    """Token-budgeted sub-batches with copy-stream H2D + async D2H == the fp32 torch encoder."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, TorchEncoder
    from codename_symbiont_amd.models.weights import load_params
    from codename_symbiont_amd.services.batcher import EmbedBatcher
    from codename_symbiont_amd.text.tokenizer import Tokenizer

    cfg = get_config("minilm-l6")
    params = load_params(cfg, seed=3, device="cpu")
    hip_enc = HipEncoder(cfg, params=params)
    ref_enc = TorchEncoder(cfg, params=params)
    tok = Tokenizer(cfg)
    rng = np.random.default_rng(0)
    words = [w for w in tok.vocab[1000:6000] if w.isalpha()]
    texts = [" ".join(rng.choice(words, size=int(rng.integers(3, 60)))) for _ in range(300)]
    batcher = EmbedBatcher(hip_enc, tok, token_budget=2048)   # forces many sub-batches
    got = batcher._encode_all(texts)
    ref = EmbedBatcher(ref_enc, tok)._encode_all(texts)
    assert got.shape == ref.shape == (300, cfg.hidden)
    cos = (got * ref).sum(1) / (np.linalg.norm(got, axis=1) * np.linalg.norm(ref, axis=1))
    assert cos.min() > 0.999, cos.min()


def test_ingest_and_search_on_gpu():
    from codename_symbiont_amd.services.api import ApiService
    from codename_symbiont_amd.services.preprocessing import PreprocessingService
    from codename_symbiont_amd.services.vector_memory import VectorMemoryService
    from codename_symbiont_amd.wire import RawTextMessage, subjects

    from helpers import broker, cpu_config, start_api, stop_api

    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url, force_cpu=False, index_capacity=1 << 16)
            pre = await PreprocessingService(cfg).start()
            vm = await VectorMemoryService(cfg).start()
            assert vm.store.shard.device.type == "cuda"
            api = ApiService(cfg)
            url, t = await start_api(api)
            sents = [f"Sentence number {i} talks about topic {i % 7} in detail." for i in range(40)]
            raw = RawTextMessage("doc-gpu", "http://example.org/gpu", " ".join(sents), 1)
            await api.nc.publish(subjects.RAW_TEXT_DISCOVERED, raw.to_json())
            for _ in range(400):
                if vm.store.count >= 40:
                    break
                await asyncio.sleep(0.05)
            assert vm.store.count == 40
            async with httpx.AsyncClient(timeout=30) as c:
                r = await c.post(url + "/api/search/semantic",
                                 json={"query_text": sents[17], "top_k": 5})
            assert r.status_code == 200, r.text
            body = r.json()
            assert body["error_message"] is None and len(body["results"]) == 5
            top = body["results"][0]
            assert top["payload"]["sentence_text"] == sents[17]
            assert top["payload"]["sentence_order"] == 17
            assert top["score"] > 0.99
            await stop_api(api, t)
            await pre.stop()
            await vm.stop()
    asyncio.run(asyncio.wait_for(main(), 300))
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("extra,debug", [([], False), (["--opt", "overlap=0"], False), ([], True),
                                         (["--mode", "embed"], False),
                                         (["--mode", "embed", "--opt", "graph=0"], False)])
def test_bench_contract_small_index(extra, debug):
    """bench.py's driver contract (one JSON line, whole-job value, step timing) on a small index,
    with and without the encode/search stream overlap."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3",
                          "--warmup", "2", "--index-rows", "2000000"] + extra,
                         capture_output=True, text=True, timeout=300, cwd=root,
                         env=dict(os.environ, SYMB_GPU_DEBUG="1" if debug else "0"))
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 1 and r["steps"] == 3 and r["warmup"] == 2
    assert r["value"] > 0 and r["higher_is_better"] is True and r["dtype"] == "bf16"
    assert abs(r["value"] - 256 * 1000.0 / r["ms_per_step"]) / r["value"] < 0.01
    # the config lists the knobs set away from their defaults (VERDICT r4 housekeeping)
    assert ("overlap" in r["config"]) is ("overlap=0" in extra)
    assert r["config"].get("encoder_hipgraph", False) is ("--mode" in extra
                                                          and "graph=0" not in extra and not debug)
    if "--mode" not in extra:   # the held-out search rate rides in the headline's line
        assert r["heldout_searches"] == 20 and r["heldout_topk_qps"] > 0
        assert "stream scan" in r["config"]["index_scan"]


@pytest.mark.gpu
def test_gpu_debug_mode_serializes_and_matches():
    """SYMB_GPU_DEBUG's launch serialization (sync + check after every kernel) leaves the
    encoder's results bit-identical."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch
    from codename_symbiont_amd.ops._ext import hip

    cfg = get_config("minilm-l6")
    enc = HipEncoder(cfg, seed=3)
    b = synthetic_batch(cfg, 8, 40, seed=4, varlen=True).to("cuda")
    ref, _ = enc.forward_packed(b)
    was = hip().debug()
    hip().set_debug(True)
    try:
        assert hip().debug()
        out, _ = enc.forward_packed(b)
    finally:
        hip().set_debug(was)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
