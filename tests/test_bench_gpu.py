"""bench.py on the GPU with a tiny model, one timed step: the default shape (one operator
per GPU) and two operator shards (the rank process + one child shard on the same GPU).
The JSON line must account for every shard's failures and report the shard layout."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("shards", [None, 2])
def test_bench_on_gpu(shards):
    extra = [] if shards is None else ["--shards", str(shards)]
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--model", "tiny-gqa4", "--steps", "1",
                        "--warmup", "1", "--batch", "16", "--max-batch", "16", "--max-tokens", "12",
                        "--prompt-tokens", "256", "--log-kb", "8", "--patterns", "100", "--kv-gb", "2", *extra],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["config"]["operator_shards_per_gpu"] == (shards or 1) and d["config"]["global_batch"] == 16
    assert d["detail"]["outcomes"] == {"ai-complete": 16}          # every shard's failures
    assert d["detail"]["decode_tokens_per_gpu"] >= 16 * 11
    assert d["value"] > 0 and d["p50_explanation_latency_ms"] > 0
    assert ("shard 1" in r.stderr) == (shards == 2)                 # the child shard ran
