"""Tokenizer for the explanation model.

If a HuggingFace ``tokenizer.json`` is available (model directory or
``OAMD_TOKENIZER``) it is used as-is. Otherwise — the normal case offline,
where no Llama-3 vocabulary files exist — a byte-level BPE is trained
deterministically on a synthetic corpus of pod-log lines and failure
explanations (``tokenizers`` library, Rust core) and cached on disk, so token
counts per log line are realistic (~3-4 bytes/token) instead of the 1 byte/token
of a raw byte fallback. Special ids (BOS/EOS) come from the model config, and
ids the trained vocabulary does not cover (a random-weight model can sample
any id < vocab_size) are folded into range for decoding.

A checkpoint tokenizer is used the way HF ``apply_chat_template`` uses it: its
own post-processor's special tokens are NOT added (Llama-3's tokenizer.json
would otherwise put a second <|begin_of_text|> in front of ours); BOS comes from
the model config (``add_bos``: Qwen2 has none), and with a chat template (the
checkpoint's ``tokenizer_config.json`` ``chat_template``, or an explicit one)
each prompt is rendered as one user turn plus the assistant generation prompt,
which also supplies BOS.
"""
from __future__ import annotations

import hashlib
import json
import os
import threading
import time
from pathlib import Path

_CACHE = Path(os.environ.get("OAMD_CACHE_DIR", Path(__file__).resolve().parent.parent / ".cache"))
_lock = threading.Lock()

_EXPLAIN_TEXT = """Root Cause: the container was terminated because it exceeded its memory limit.
Evidence: the log shows OOMKilled shortly after the heap grew past the configured maximum.
Fix: raise resources.limits.memory or reduce the JVM heap with -Xmx so the process fits the cgroup.
Root Cause: the application could not reach its database; connections were refused.
Evidence: repeated Connection refused errors followed by retrying in 5 seconds.
Fix: verify the database service, its endpoints and network policies, and add a readiness dependency.
Root Cause: a required configuration value or secret is missing.
Fix: define the environment variable in the Deployment or mount the referenced Secret.
The pod entered CrashLoopBackOff after the liveness probe failed repeatedly.
Consider increasing initialDelaySeconds, checking the probe path, and reviewing recent deployments.
"""


def _corpus(n_lines: int = 40000):
    from operator_amd.patterns.synth import CATALOG, LogFactory

    fac = LogFactory(n_patterns=200, seed=123, pool_lines=4096)
    for line in fac.pool:
        yield line.decode()
    for c in CATALOG:
        yield c[6]
    for pid, ex in list(fac.examples.items())[:2000]:
        for e in ex:
            yield e
    for _ in range(50):
        for line in _EXPLAIN_TEXT.splitlines():
            yield line


def load_chat_template(spec: str | None, model_dir: str | None) -> str | None:
    """Resolve ``engine.chat_template``: "none"/"" -> None; "auto" -> the checkpoint's
    ``tokenizer_config.json`` chat_template (None without one); a path -> that file;
    anything else is the Jinja template itself."""
    if not spec or spec == "none":
        return None
    if spec == "auto":
        if not model_dir:
            return None
        f = os.path.join(model_dir, "tokenizer_config.json")
        if not os.path.exists(f):
            return None
        with open(f) as fh:
            t = json.load(fh).get("chat_template")
        if isinstance(t, list):  # named templates: take "default"
            t = next((x.get("template") for x in t if x.get("name") == "default"), None)
        return t or None
    if os.path.exists(spec):
        with open(spec) as fh:
            return fh.read()
    return spec


def _compile_template(src: str):
    from jinja2.exceptions import TemplateError
    from jinja2.sandbox import ImmutableSandboxedEnvironment

    def raise_exception(msg):
        raise TemplateError(msg)

    env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
    env.globals["raise_exception"] = raise_exception
    env.globals["strftime_now"] = lambda fmt: time.strftime(fmt)
    return env.from_string(src)


class Tokenizer:
    def __init__(self, vocab_limit: int, bos_id: int, eos_id: int, path: str | None = None,
                 add_bos: bool = True, chat_template: str | None = None):
        import tokenizers

        self.bos_id, self.eos_id = bos_id, eos_id
        self.add_bos = add_bos and bos_id >= 0
        path = path or os.environ.get("OAMD_TOKENIZER")
        self.from_checkpoint = bool(path and os.path.exists(path))
        if self.from_checkpoint:
            self.tk = tokenizers.Tokenizer.from_file(path)
        else:
            self.tk = self._trained(min(32000, max(256 + 8, vocab_limit - 16)))
        self.n_vocab = self.tk.get_vocab_size()
        self.chat = _compile_template(chat_template) if chat_template else None
        if self.chat is not None:
            tok = lambda i: (self.tk.id_to_token(i) or "") if i >= 0 else ""  # noqa: E731
            self._chat_vars = {"bos_token": tok(bos_id), "eos_token": tok(eos_id), "add_generation_prompt": True}

    def render_chat(self, text: str) -> str:
        """One user turn + the assistant generation prompt, through the chat template."""
        return self.chat.render(messages=[{"role": "user", "content": text}], **self._chat_vars)

    @staticmethod
    def _trained(vocab: int):
        import tokenizers
        from tokenizers import decoders, models, pre_tokenizers, trainers

        key = hashlib.sha1(f"bpe-v1-{vocab}".encode()).hexdigest()[:12]
        f = _CACHE / f"tokenizer-{key}.json"
        with _lock:
            if f.exists():
                return tokenizers.Tokenizer.from_file(str(f))
            tk = tokenizers.Tokenizer(models.BPE())
            tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
            tk.decoder = decoders.ByteLevel()
            tr = trainers.BpeTrainer(vocab_size=vocab, show_progress=False,
                                     initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
            tk.train_from_iterator(_corpus(), trainer=tr)
            _CACHE.mkdir(parents=True, exist_ok=True)
            tmp = f.with_suffix(f".{os.getpid()}.tmp")
            tk.save(str(tmp))
            os.replace(tmp, f)
            return tk

    def encode_chat(self, messages: list[dict]) -> list[int]:
        """Token ids of a chat (``[{"role", "content"}, ...]``) ending in the assistant's
        turn: through the checkpoint's chat template when there is one, else as plain
        ``role: content`` lines after BOS."""
        msgs = [{"role": str(m.get("role", "user")), "content": str(m.get("content") or "")} for m in messages]
        if self.chat is not None:
            text = self.chat.render(messages=msgs, **self._chat_vars)
            return self.tk.encode(text, add_special_tokens=False).ids
        text = "".join(f"{m['role']}: {m['content']}\n" for m in msgs) + "assistant:"
        return ([self.bos_id] if self.add_bos else []) + self.tk.encode(text, add_special_tokens=False).ids

    def encode_text(self, text: str) -> list[int]:
        """Token ids of a raw completion prompt (BOS when the model has one; no chat template)."""
        return ([self.bos_id] if self.add_bos else []) + self.tk.encode(text, add_special_tokens=False).ids

    def encode(self, text: str, bos: bool = True) -> list[int]:
        return self.encode_batch([text], bos)[0]

    def encode_batch(self, texts: list[str], bos: bool = True) -> list[list[int]]:
        """Prompt token ids. ``bos`` prepends the config's BOS (when the model has one);
        with a chat template the template places BOS and the turn markers instead."""
        if self.chat is not None:
            return [e.ids for e in self.tk.encode_batch([self.render_chat(t) for t in texts],
                                                        add_special_tokens=False)]
        pre = [self.bos_id] if (bos and self.add_bos) else []
        return [pre + e.ids for e in self.tk.encode_batch(texts, add_special_tokens=False)]

    def _keep(self, ids: list[int]) -> list[int]:
        n = self.n_vocab
        return [i % n for i in ids if i != self.bos_id and i != self.eos_id]

    def decode(self, ids: list[int]) -> str:
        return self.tk.decode(self._keep(ids), skip_special_tokens=self.from_checkpoint)

    def decode_batch(self, seqs: list[list[int]]) -> list[str]:
        """``decode`` of many sequences in one call (the Rust core runs them in
        parallel without the GIL)."""
        return self.tk.decode_batch([self._keep(x) for x in seqs], skip_special_tokens=self.from_checkpoint)

    # ------------------------------------------------------------------ incremental decoding
    _bytes = None

    def byte_table(self) -> list[bytes] | None:
        """id -> the bytes it stands for, when decoding is a plain byte-level BPE (decode(ids)
        == the UTF-8 ('replace') text of the concatenated bytes of the kept ids); None for any
        other decoder. Checked once against ``decode`` on random sequences, so streaming
        detokenization (``feed`` / ``text_of``) is used only where it is exact."""
        if self._bytes is None:
            self._bytes = self._build_byte_table() or False
        return self._bytes or None

    def _build_byte_table(self):
        bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + \
            list(range(ord("\xae"), ord("\xff") + 1))
        cs, n = bs[:], 0
        for b in range(256):
            if b not in bs:
                bs.append(b)
                cs.append(256 + n)
                n += 1
        u2b = {chr(c): b for b, c in zip(bs, cs)}
        # added tokens are decoded as their literal content, not through the byte-level
        # alphabet; special ones (a checkpoint's 256 Llama-3 <|...|> ids) are dropped by
        # decode(skip_special_tokens=True), so they stand for no bytes at all
        added = {}
        for i, at in self.tk.get_added_tokens_decoder().items():
            added[i] = b"" if (at.special and self.from_checkpoint) else at.content.encode("utf-8")
        table = []
        for i in range(self.n_vocab):
            if i in added:
                table.append(added[i])
                continue
            t = self.tk.id_to_token(i)
            if t is None or any(c not in u2b for c in t):
                return None
            table.append(bytes(u2b[c] for c in t))
        import random
        rng = random.Random(7)
        for k in range(64):
            ids = [rng.randrange(0, self.n_vocab) for _ in range(rng.randrange(1, 300))]
            if k % 2:   # also ids past the vocabulary, BOS/EOS
                ids += [self.n_vocab + 5, self.eos_id, self.bos_id, 2 * self.n_vocab + 1]
            kept = self._keep(ids)
            if b"".join(table[j] for j in kept).decode("utf-8", "replace") != self.decode(ids):
                return None
        return table

    def feed(self, buf: bytearray, ids: list[int]) -> None:
        """Append the bytes of ``ids`` (the same ids ``decode`` keeps) to ``buf``."""
        table, n, bos, eos = self._bytes, self.n_vocab, self.bos_id, self.eos_id
        buf += b"".join([table[i % n] for i in ids if i != bos and i != eos])

    @staticmethod
    def text_of(buf: bytearray) -> str:
        return buf.decode("utf-8", "replace")
