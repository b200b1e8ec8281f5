"""Native build of the MI355X classification path (in-tree, no JIT cache).

  odp_amd/libmi_cls.so   hipcc --offload-arch=gfx950: HIP kernels + mi_cls.h C ABI
  odp_amd/libodp_cls.so  gcc: ODP classification control plane (odp_cls_api.h),
                         linked against libmi_cls.so (rpath $ORIGIN)
"""
from __future__ import annotations

import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "odp_amd")
SRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(force: bool = False, out_dir: str = PKG, defines=()) -> list[str]:
    """Build both libraries into out_dir (default: in-tree).  ``defines``
    (e.g. ["WIN=64"]) builds a kernel variant for A/B measurement."""
    hdrs = [os.path.join(INC, h) for h in ("mi_cls.h", "odp_cls_api.h")]
    mi_src = os.path.join(SRC, "mi_cls.hip")
    os.makedirs(out_dir, exist_ok=True)
    mi_so = os.path.join(out_dir, "libmi_cls.so")
    odp_src = os.path.join(SRC, "odp_cls.c")
    odp_so = os.path.join(out_dir, "libodp_cls.so")
    built = []
    if force or defines or _stale(mi_so, [mi_src] + hdrs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wall", "-I", INC] + [f"-D{d}" for d in defines] + ["-o", mi_so, mi_src])
        built.append(mi_so)
    if force or _stale(odp_so, [odp_src, mi_so] + hdrs):
        _run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-fPIC", "-shared", "-I", INC,
              "-o", odp_so, odp_src, "-L", out_dir, "-lmi_cls", "-Wl,-rpath,$ORIGIN",
              "-lpthread"])
        built.append(odp_so)
    return built


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 2:   # python -m odp_amd._build OUT_DIR DEF=1 ...
        print(build(force=True, out_dir=sys.argv[1], defines=sys.argv[2:]))
    else:
        print(build(force=True))
