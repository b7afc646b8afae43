"""Read back HDF5 files in tests through the image's `h5dump` (HDF5 1.10 CLI),
independently of the writer under test (libmgic_io).  h5py is not installed."""
import os
import re
import shutil
import subprocess
import tempfile

import numpy as np


def h5dump_path() -> str:
    p = shutil.which("h5dump") or "/opt/conda/bin/h5dump"
    if not os.path.exists(p):
        raise FileNotFoundError("h5dump not found (expected /opt/conda/bin/h5dump)")
    return p


def _run(args):
    return subprocess.run([h5dump_path()] + args, check=True, capture_output=True,
                          text=True).stdout


def contents(fname):
    """{path: 'group' | 'dataset'}"""
    out = {}
    for line in _run(["-n", fname]).splitlines():
        m = re.match(r"\s*(group|dataset)\s+(\S+)", line)
        if m:
            out[m.group(2)] = m.group(1)
    return out


def attr(fname, path):
    """A scalar attribute: str, int / float, or a tuple of ints (compound)."""
    txt = _run(["-a", path, fname])
    data = txt[txt.index("DATA {"):]
    s = re.search(r'"(.*)"', data)
    if s and "H5T_STRING" in txt:
        return s.group(1)
    nums = re.findall(r"-?\d+(?:\.\d*)?(?:e[-+]?\d+)?", data.split("(0):", 1)[1])
    if "H5T_COMPOUND" in txt:
        return tuple(int(v) for v in nums)
    v = nums[0]
    return float(v) if ("H5T_IEEE" in txt) else int(v)


def dataset(fname, path, dtype):
    """The raw little-endian contents of a dataset as a numpy array."""
    with tempfile.TemporaryDirectory() as d:
        b = os.path.join(d, "x.bin")
        _run(["-d", path, "-b", "LE", "-o", b, fname])
        return np.fromfile(b, dtype=dtype)


def boxes(fname, level):
    """The "boxes" dataset of a level as a list of 6-tuples (text dump: the
    binary dump does not take compound types)."""
    txt = _run(["-d", f"/level_{level}/boxes", fname])
    data = txt[txt.index("DATA {") + 6:]
    nums = [int(v) for v in re.findall(r"(?<![(\d])-?\d+(?![\d)])", data)]
    return [tuple(nums[i:i + 6]) for i in range(0, len(nums), 6)]
