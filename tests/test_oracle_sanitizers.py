"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY 5:
sanitizers on host code). `make -C oracle asan` builds the same md_oracle.c with
-fsanitize=address,undefined -fno-sanitize-recover=all; a child Python process
with the ASan runtime preloaded loads it (MDO_LIB) and reruns the reference's
known answers, then full deconvolutions (single, and a 4-thread batch over
spectra) whose results must equal the normal build's bit for bit. Any report
aborts the child."""
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

ORACLE = os.path.join(ROOT, "oracle")

CHILD = r"""
import os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "metabodecon-rust_amd")]
import numpy as np
import oracle
from tests.golden.cases import load_case
names = ["sim_01", "blood_01", "blood_01_water", "sim_01_detector_only"]
out = []
for n in names:
    x, y, sb, st, ign = load_case(n)
    r = oracle.deconvolute(x, y, sb, st, ign)
    out.append((r.status, r.params.tobytes().hex()[:4096], float(r.mse).hex()))
x, y, sb, _, _ = load_case("blood_02")
ys = np.stack([y] * 4)
st, cnt, params, mse = oracle.deconvolute_batch(x, ys, [sb] * 4, threads=4)
out.append((st.tolist(), cnt.tolist(), params[0, : cnt[0]].tobytes().hex()[:4096],
            [float(m).hex() for m in mse]))
print(repr(out))
"""


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], capture_output=True,
                          text=True, env=env, timeout=600, cwd=ROOT)


@pytest.fixture(scope="module")
def asan_env():
    r = subprocess.run(["make", "-s", "-C", ORACLE, "asan"], capture_output=True, text=True)
    if r.returncode:
        pytest.skip("sanitizer build failed: " + r.stderr[-500:])
    libs = [subprocess.run(["gcc", f"-print-file-name={n}"], capture_output=True,
                           text=True).stdout.strip() for n in ("libasan.so", "libubsan.so")]
    if not all(os.path.isabs(p) and os.path.exists(p) for p in libs):
        pytest.skip("no ASan/UBSan runtime")
    return {"LD_PRELOAD": ":".join(libs), "MDO_LIB": os.path.join(ORACLE, "libmd_oracle_asan.so"),
            "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
            "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}


def test_known_answers_under_sanitizers(asan_env):
    env = dict(os.environ, **asan_env)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle_known_answers.py")],
                       capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_deconvolutions_under_sanitizers_match_normal_build(asan_env):
    sanitized = _run(asan_env)
    assert sanitized.returncode == 0, sanitized.stderr[-3000:]
    assert "runtime error" not in sanitized.stderr
    normal = _run({})
    assert normal.returncode == 0, normal.stderr[-3000:]
    assert sanitized.stdout == normal.stdout
