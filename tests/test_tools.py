"""The measurement tools still run against the current tree: every
tools/*.py answers --help on a CPU box without touching a GPU (argument parsing
comes before any engine import), and every tools/*.sh parses (bash -n). Each tool's
own GPU work is exercised on the GPU box by the sessions that use it
(tools/gpu_run.sh)."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY_TOOLS = sorted(glob.glob(os.path.join(ROOT, "tools", "*.py")))
SH_TOOLS = sorted(glob.glob(os.path.join(ROOT, "tools", "*.sh")))


@pytest.mark.parametrize("path", PY_TOOLS, ids=os.path.basename)
def test_tool_help(path):
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, path, "--help"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, (path, r.stderr[-2000:])
    assert r.stdout.startswith("usage:"), (path, r.stdout[:200])


@pytest.mark.parametrize("path", SH_TOOLS, ids=os.path.basename)
def test_shell_tool_parses(path):
    r = subprocess.run(["bash", "-n", path], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, (path, r.stderr)


def test_gen_chain_asm_help_writes_nothing():
    inc = os.path.join(ROOT, "metabodecon-rust_amd", "csrc", "mdg_chain_asm.inc")
    before = os.stat(inc).st_mtime_ns
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_chain_asm.py"), "--help"],
                   capture_output=True, timeout=60, check=True)
    assert os.stat(inc).st_mtime_ns == before


UBENCH = sorted(glob.glob(os.path.join(ROOT, "tools", "ubench", "*.hip")))
HIPCC = "/opt/rocm/bin/hipcc"
HIP_FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
             "-DMDG_DIAG", "-fsyntax-only"]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("path", UBENCH, ids=os.path.basename)
def test_ubench_source_compiles_against_the_engine(path):
    """The microbenchmarks include the engine's kernel source: an API change there
    (round 5: the launchers take the context's EngineSwitches) must not leave them
    stale."""
    r = subprocess.run([HIPCC] + HIP_FLAGS + [path], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_ubench_check_has_power(tmp_path):
    bad = tmp_path / "stale.hip"
    bad.write_text('#include "%s"\nusing namespace mdg;\n'
                   'void f(const BatchArgs& a, const Workspace& w) { launch_fit_sup(a, w, 24, 0, 0); }\n'
                   % os.path.join(ROOT, "metabodecon-rust_amd", "csrc", "mdg_kernels.hip"))
    r = subprocess.run([HIPCC] + HIP_FLAGS + [str(bad)], capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
