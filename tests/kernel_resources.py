"""Per-kernel resource metadata of a built HIP library (CPU only, no GPU).

Reads the gfx950 code objects embedded in a shared library's `.hip_fatbin`
section (one clang offload bundle per translation unit), and from each the
AMDGPU metadata note (`llvm-readelf --notes`): per kernel its private segment
(scratch bytes per lane), VGPR spill count and VGPR count.  Used by
tests/test_kernel_resources.py against the committed budget
tests/kernel_budget.json, and runnable by hand:

    python3 tests/kernel_resources.py [motionestimation_amd/lib/libme_hip.so]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def tools_present():
    return all(os.access(os.path.join(LLVM, t), os.X_OK) for t in ("llvm-objcopy", "llvm-readelf"))


def _fatbin(lib):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "fatbin.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={out}", lib,
                        os.path.join(td, "discard.o")], check=True, capture_output=True)
        with open(out, "rb") as f:
            return f.read()


def code_objects(lib, arch="gfx950"):
    """The `arch` code objects (ELF bytes) of every offload bundle in `lib`."""
    data = _fatbin(lib)
    objs = []
    pos = data.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", data, pos + len(MAGIC))
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if triple.endswith("--" + arch) and size:
                objs.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + len(MAGIC))
    return objs


_FIELDS = ("name", "private_segment_fixed_size", "vgpr_spill_count", "vgpr_count", "sgpr_spill_count")


def kernels(lib, arch="gfx950"):
    """{mangled kernel name: {field: int}} over every code object of `lib`."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for i, obj in enumerate(code_objects(lib, arch)):
            path = os.path.join(td, f"co{i}.o")
            with open(path, "wb") as f:
                f.write(obj)
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", path], check=True,
                                   capture_output=True, text=True).stdout
            # one kernel per "  - .agpr_count" list item of amdhsa.kernels
            for item in re.split(r"\n  - ", notes)[1:]:
                rec = {}
                for fld in _FIELDS:
                    m = re.search(r"^\s*\.?%s:\s+(\S+)" % fld, item, re.M)
                    if m:
                        rec[fld] = m.group(1) if fld == "name" else int(m.group(1))
                if "name" in rec and "private_segment_fixed_size" in rec:
                    out[rec.pop("name")] = rec
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return dict(zip(names, r.stdout.splitlines()))
    except (OSError, subprocess.CalledProcessError):
        return {n: n for n in names}


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "motionestimation_amd", "lib", "libme_hip.so")
    ks = kernels(lib)
    dm = demangle(sorted(ks))
    for n in sorted(ks):
        r = ks[n]
        print(f"{r['private_segment_fixed_size']:4d} B scratch  {r['vgpr_spill_count']:3d} VGPR spills  "
              f"{r['vgpr_count']:4d} VGPRs  {dm[n]}")
