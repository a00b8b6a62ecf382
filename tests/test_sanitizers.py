"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer.

The pattern compiler, doc packer (multi-threaded memcpy into a staging buffer)
and event scorer are rebuilt with -fsanitize=address,undefined into a temp dir
and driven with randomized inputs in a child Python that preloads libasan; any
report aborts the child and fails the test. (GPU-side sanitizers are not
available on the MI355X pool; the kernels are covered by the fp32 reference
tests instead.)"""
import os
import subprocess
import sys
import textwrap

import pytest

DRIVER = textwrap.dedent(r"""
    import random, sys, numpy as np
    sys.path.insert(0, sys.argv[1])
    import _patterns as P
    rnd = random.Random(0)
    alpha = b"abcdefghijklmnopqrstuvwxyzABCXYZ0123456789 :_-."
    for trial in range(40):
        nf = rnd.randint(1, 300)
        factors = list({bytes(rnd.choice(alpha) for _ in range(rnd.randint(1, 64))) for _ in range(nf)})
        d = P.compile_dfa(factors)
        assert d["num_states"] >= 1
        docs = [bytes(rnd.choice(alpha + b"\n") for _ in range(rnd.randint(0, 5000))) for _ in range(rnd.randint(1, 30))]
        seg = rnd.choice([64, 256, 1024])
        total_bytes, first = P.plan_docs([len(x) for x in docs], seg)
        buf = np.zeros(total_bytes, dtype=np.uint8)
        P.pack_docs(docs, first, seg, buf.ctypes.data, rnd.randint(1, 8))
        for i, x in enumerate(docs):
            o = first[i] * seg
            assert bytes(buf[o:o + len(x)]) == x and buf[o + len(x)] == 0
        n = rnd.randint(0, 500)
        nm, npat = 20, 10
        hd = [rnd.randrange(len(docs)) for _ in range(n)]
        hm = [rnd.randrange(nm) for _ in range(n)]
        hl = [rnd.randrange(200) for _ in range(n)]
        prim = [rnd.randrange(nm) for _ in range(npat)]
        sec = [[rnd.randrange(nm) for _ in range(rnd.randint(0, 3))] for _ in range(npat)]
        res = P.score_events(hd, hm, hl, len(docs), prim, [rnd.random() for _ in range(npat)],
                             [rnd.randrange(5) for _ in range(npat)], sec,
                             [[rnd.random() for _ in s] for s in sec], [[rnd.randint(0, 20) for _ in s] for s in sec], nm)
        assert len(res) == len(docs)
    for bad in ([b""], [b"x" * 65], [b"a\nb"], [b"a\x00b"]):
        try:
            P.compile_dfa(bad)
        except ValueError:
            pass
        else:
            raise AssertionError(bad)
    print("sanitized ok")
""")


def _lib(name):
    for cc in ("g++", "gcc"):
        try:
            p = subprocess.run([cc, f"-print-file-name={name}"], capture_output=True, text=True, check=True)
        except (OSError, subprocess.CalledProcessError):
            continue
        path = p.stdout.strip()
        if os.path.isabs(path) and os.path.exists(path):
            return path
    return None


def _libasan():
    asan = _lib("libasan.so")
    # libstdc++ must be loaded when ASan initialises, or its __cxa_throw
    # interceptor has nothing to forward to (python itself is not C++)
    cxx = _lib("libstdc++.so.6") or _lib("libstdc++.so")
    return f"{asan} {cxx}" if asan and cxx else asan


def test_host_cpp_under_asan_ubsan(tmp_path):
    asan = _libasan()
    if asan is None:
        pytest.skip("libasan not available")
    from operator_amd import _build

    _build.build_patterns(force=True, out_dir=tmp_path, sanitize=True)
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-c", DRIVER, str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "sanitized ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
