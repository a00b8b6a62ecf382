"""Model-weight cache: one rank's ready-to-run shard (TP-sliced, gate|up interleaved,
fp8-quantized) as a safetensors file, memory-mapped back at start-up.

SURVEY.md §5.4 ("an optional ... model-weight mmap cache"; the engine is otherwise
stateless across restarts). The reference has no weights (its LLM is external,
J/service/AIInterfaceRestClient.java:37-39); here a restarted engine skips the HF
read + re-shard + re-quantize (or the random init) and maps the shard it had: the
file is read by the OS's page cache straight into the device tensors
(``safe_open(device=...)``), no pickle, nothing executed from the file.

The file name carries a key over everything that shapes the shard: architecture,
TP rank / world, compute dtype, weight dtype, gate|up interleave, the source
(HF files' sizes + mtimes, or the random-init seed) and the source text of the
code that builds the layout (``layout_version``), so a stale shard is never loaded. Writes go to a temporary name and are renamed into place (a crash mid-write
leaves no half file under the real name).
"""
from __future__ import annotations

import dataclasses
import glob
import hashlib
import json
import logging
import os

import torch

log = logging.getLogger(__name__)

FORMAT = 1
LAYER_FIELDS = ("wqkv", "wo", "wgu", "wd", "attn_norm", "mlp_norm", "sqkv", "so", "sgu", "sd", "bqkv")


def source_id(model_path: str | None, seed: int) -> str:
    """What the weights are made from: the checkpoint files (name, size, mtime) or the seed."""
    if not model_path:
        return f"random:{seed}"
    files = sorted(glob.glob(os.path.join(model_path, "*.safetensors")) + [os.path.join(model_path, "config.json")])
    parts = []
    for f in files:
        if os.path.exists(f):
            st = os.stat(f)
            parts.append(f"{os.path.basename(f)}:{st.st_size}:{int(st.st_mtime)}")
    return "hf:" + os.path.abspath(model_path) + ":" + ",".join(parts)


# the code that lays a shard out: TP slicing, QKV packing, gate|up interleave, fp8 scale
# rounding, the random init. Its source text is part of the key, so an edit to any of it
# misses every cache file written before the edit instead of mapping a stale layout back.
LAYOUT_FUNCS = ("init_random", "_randn", "_quantize_layer", "_shard_layer", "split_gate_up", "load_hf")


def layout_version(model_cls=None) -> str:
    import inspect

    from operator_amd import ops

    if model_cls is None:
        from .llama import LlamaModel as model_cls
    src = "".join(inspect.getsource(getattr(model_cls, f)) for f in LAYOUT_FUNCS)
    src += inspect.getsource(ops.interleave_gate_up) + inspect.getsource(ops.quantize_fp8)
    return hashlib.sha256(src.encode()).hexdigest()[:16]


def cache_path(cache_dir: str, model, source: str) -> str:
    blob = json.dumps({"format": FORMAT, "layout": layout_version(type(model)), "cfg": dataclasses.asdict(model.cfg),
                       "tp": [model.tp.rank, model.tp.world],
                       "dtype": str(model.dtype), "fp8": model.fp8, "gu_block": model.gu_block, "source": source},
                      sort_keys=True, default=str)
    key = hashlib.sha256(blob.encode()).hexdigest()[:24]
    return os.path.join(cache_dir, f"{model.cfg.name}-{key}-r{model.tp.rank}of{model.tp.world}.safetensors")


def save(model, path: str) -> None:
    from safetensors.torch import save_file

    t = {"embed": model.embed, "final_norm": model.final_norm, "lm_head": model.lm_head}
    for i, lw in enumerate(model.layers):
        for f in LAYER_FIELDS:
            v = getattr(lw, f)
            if v is not None:
                t[f"l{i}.{f}"] = v
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    # the tied lm_head may share storage with embed: safetensors refuses aliases
    save_file({k: v.detach().contiguous().cpu().clone() if k == "lm_head" else v.detach().contiguous().cpu()
               for k, v in t.items()}, tmp, metadata={"format": str(FORMAT), "layers": str(len(model.layers))})
    os.replace(tmp, path)


def load(model, path: str) -> None:
    """Fill ``model``'s weights from a cache file written by ``save`` for the same key."""
    from safetensors import safe_open

    from .llama import LayerWeights

    dev = str(model.device)
    with safe_open(path, framework="pt", device=dev) as f:
        n = int(f.metadata()["layers"])
        names = set(f.keys())
        model.embed = f.get_tensor("embed")
        model.final_norm = f.get_tensor("final_norm")
        model.lm_head = f.get_tensor("lm_head")
        layers = []
        for i in range(n):
            kw = {fld: (f.get_tensor(f"l{i}.{fld}") if f"l{i}.{fld}" in names else None) for fld in LAYER_FIELDS}
            layers.append(LayerWeights(**kw))
        model.layers = layers
    if model.device.type == "cuda":
        torch.cuda.synchronize(model.device)


def load_or_build(model, cache_dir: str | None, model_path: str | None, seed: int) -> str:
    """Weights from the cache when a file for this exact shard exists, else built (HF
    load or random init) and written to the cache. Returns 'hit', 'miss' or 'off'."""
    build = (lambda: model.load_hf(model_path)) if model_path else (lambda: model.init_random(seed))
    if not cache_dir:
        build()
        return "off"
    path = cache_path(cache_dir, model, source_id(model_path, seed))
    if os.path.exists(path):
        try:
            load(model, path)
            log.info("model weights mapped from the cache: %s", path)
            return "hit"
        except Exception as e:  # noqa: BLE001 - a damaged file is rebuilt
            log.warning("weight cache %s unreadable (%s); rebuilding", path, e)
    build()
    try:
        save(model, path)
        log.info("model weights cached: %s", path)
    except OSError as e:
        log.warning("could not write the weight cache %s: %s", path, e)
    return "miss"
