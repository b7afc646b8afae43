"""The process-wide HIP runtime guard (mg_ic_code_amd/_lib.py
check_single_hip_runtime): torch bundles its own libamdhip64, and a process
that loads libmgic.so (bound to /opt/rocm's by soname) before torch holds two
runtimes, which corrupt each other's heap at exit.  CPU tests: no GPU call is
made (the check runs before any)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mg_ic_code_amd  # noqa: E402,F401
from mg_ic_code_amd import _lib  # noqa: E402


def test_this_process_maps_one_hip_runtime():
    imgs = _lib.hip_runtime_images()
    assert len(imgs) <= 1, imgs
    _lib.check_single_hip_runtime()


def test_second_runtime_fails_loudly():
    # torch imported AFTER the library (preload disabled): the next Comm()
    # raises with both paths named instead of running on to the exit abort
    code = ("import mg_ic_code_amd as mg\n"
            "import torch\n"
            "mg.Comm()\n")
    env = dict(os.environ, MGIC_NO_TORCH_PRELOAD="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0
    assert "two HIP runtimes in one process" in r.stderr, r.stderr[-2000:]


def test_default_preload_keeps_one_runtime():
    # the default: importing the library first still imports torch before
    # libmgic.so, so torch imported afterwards adds nothing
    code = ("import mg_ic_code_amd\n"
            "import torch\n"
            "from mg_ic_code_amd._lib import hip_runtime_images\n"
            "print(len(hip_runtime_images()))\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] in ("0", "1")
