"""The C-ABI's host code under AddressSanitizer (SURVEY §5 "-fsanitize=address host build of the
C-ABI"): `make -C .../csrc asan` builds build/asan/libdsvt_asan.so with capi.hip's host side
instrumented (argument validation, workspace sizing, the error string); this runs the CPU C-ABI
tests (tests/test_capi_symbols.py: symbol table, arity, validation before any launch) against it
in a child process with the clang ASan runtime preloaded.  CPU only; GPU sanitizers are not
available on this pool.  Skipped when the ASan library or runtime is absent."""
import glob
import os
import subprocess
import sys

import pytest

from conftest import ROOT

ASAN_LIB = os.path.join(ROOT, "dino-video-summarization-transformer_amd", "csrc", "build", "asan", "libdsvt_asan.so")


def _runtime():
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


def test_capi_validation_under_asan():
    rt = _runtime()
    if not os.path.exists(ASAN_LIB) or rt is None:
        pytest.skip("host-ASan C-ABI library or clang ASan runtime not present (make -C csrc asan)")
    out = subprocess.run(["nm", "-D", ASAN_LIB], capture_output=True, text=True).stdout
    assert "__asan_report" in out, "libdsvt_asan.so is not instrumented"
    env = dict(os.environ, LD_PRELOAD=rt, DSVT_LIB=ASAN_LIB,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_capi_symbols.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in r.stderr, r.stdout[-2000:] + r.stderr[-4000:]
    assert " passed" in r.stdout
