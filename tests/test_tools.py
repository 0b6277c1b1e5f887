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
