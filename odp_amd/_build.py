"""Native build of the MI355X classification path (in-tree, no JIT cache).

  odp_amd/libmi_cls.so   hipcc --offload-arch=gfx950: HIP kernels + mi_cls.h C ABI
  odp_amd/mi_cls_jitc    g++ over hipRTC: compiles program-specialised kernels,
                         started by libmi_cls.so as a child process
  odp_amd/libodp_cls.so  gcc: the ODP library of this build -- classification
                         control plane (odp_cls_api.h) + runtime subset and
                         packet I/O (odp_rt.h), linked against libmi_cls.so
  odp_amd/libodph.so     gcc: the ODP helper subset (odp/helper/odph_api.h)
  examples/_bin/odp_classifier
                         the reference's example/classifier/odp_classifier.c,
                         compiled UNCHANGED from /root/reference against these
                         headers and libraries (only when the reference tree is
                         present, i.e. in the build container; the binary travels)
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
    odp_srcs = [os.path.join(SRC, f) for f in ("odp_cls.c", "odp_rt.c", "odp_pktio.c")]
    odp_so = os.path.join(out_dir, "libodp_cls.so")
    odph_src = os.path.join(SRC, "odph.c")
    odph_so = os.path.join(out_dir, "libodph.so")
    rt_hdrs = hdrs + [os.path.join(INC, "odp_rt.h"), os.path.join(INC, "odp_api.h"),
                      os.path.join(INC, "odp", "helper", "odph_api.h"),
                      os.path.join(SRC, "odp_rt_internal.h")]
    built = []
    mi_hdr = os.path.join(SRC, "mi_cls_dev.h")
    k_srcs = [os.path.join(SRC, f"mi_cls_k{w}.hip") for w in (4, 8, 12, 16, "f", "f12", "f16", "c4",
                                                              "c16", "d")]
    if force or defines or _stale(mi_so, [mi_src, mi_hdr] + k_srcs + hdrs + [__file__]):
        # one translation unit per block shape + the host code, compiled in
        # parallel (the kernel instantiations dominate the build time)
        import concurrent.futures as cf
        import tempfile
        tmp = tempfile.mkdtemp(prefix="mi_cls_obj_")
        flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I", INC,
                 "-I", SRC, "-I", tmp] + [f"-D{d}" for d in defines]
        write_src_inc(os.path.join(tmp, "mi_cls_src.inc"), defines)
        objs = []
        jobs = []
        # MI_CLS_ONLY=kf,k4 (variant builds only): compile just those kernel
        # translation units; the others become -ENOSYS stubs (mi_cls_dev.h)
        only = os.environ.get("MI_CLS_ONLY", "") if defines else ""
        keep = {f"mi_cls_{k}.hip" for k in only.split(",") if k}
        for src in [mi_src] + k_srcs:
            obj = os.path.join(tmp, os.path.basename(src) + ".o")
            objs.append(obj)
            stub = ["-DMI_CLS_STUB"] if keep and src != mi_src and \
                os.path.basename(src) not in keep else []
            jobs.append([HIPCC] + flags + stub + ["-c", "-o", obj, src])
        with cf.ThreadPoolExecutor(max_workers=len(jobs)) as ex:
            list(ex.map(_run, jobs))
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", mi_so] + objs)
        shutil.rmtree(tmp, ignore_errors=True)
        built.append(mi_so)
    # the program-specialised kernels' compiler, run as a child process of
    # libmi_cls.so (mi_cls.hip spec_compile): host code over hipRTC
    jitc_src = os.path.join(SRC, "mi_cls_jitc.cpp")
    jitc = os.path.join(out_dir, "mi_cls_jitc")
    if force or _stale(jitc, [jitc_src]):
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
              "-o", jitc, jitc_src, "-L", "/opt/rocm/lib", "-lhiprtc", "-Wl,-rpath,/opt/rocm/lib"])
        built.append(jitc)
    if force or _stale(odp_so, odp_srcs + [mi_so] + rt_hdrs):
        _run(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-fPIC", "-ftls-model=initial-exec",
              "-shared", "-I", INC, "-o", odp_so] + odp_srcs + ["-L", out_dir, "-lmi_cls", "-Wl,-rpath,$ORIGIN",
                                          "-lpthread"])
        built.append(odp_so)
    if force or _stale(odph_so, [odph_src, odp_so] + rt_hdrs):
        _run(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-fPIC", "-shared", "-I", INC,
              "-o", odph_so, odph_src, "-L", out_dir, "-lodp_cls", "-Wl,-rpath,$ORIGIN",
              "-lpthread"])
        built.append(odph_so)
    if out_dir == PKG:
        for b in (build_example(force), build_test_drivers(force)):
            if b:
                built.append(b)
    return built


def write_src_inc(path, defines=()):
    """The kernel sources as C string literals for hipRTC (program-specialised
    kernels, mi_cls.hip): mi_cls.h, mi_cls_dev.h and the build's -D options,
    so a specialised kernel is compiled from exactly the code of this build."""
    def lit(name, text):
        assert ")MICLS\"" not in text
        return f'static const char {name}[] = R"MICLS({text})MICLS";\n'
    with open(os.path.join(INC, "mi_cls.h")) as f:
        h = f.read()
    with open(os.path.join(SRC, "mi_cls_dev.h")) as f:
        dev = f.read()
    defs = ", ".join(f'"-D{d}"' for d in defines)
    with open(path, "w") as f:
        f.write(lit("mi_cls_src_h", h) + lit("mi_cls_src_dev", dev) +
                f"static const char *const mi_cls_src_defs[] = {{ {defs}{', ' if defs else ''}nullptr }};\n"
                f'static const char mi_cls_src_arch[] = "{ARCH}";\n')


TEST_BIN = os.path.join(ROOT, "tests", "_bin")


def build_test_drivers(force: bool = False):
    """Test-only C drivers of the runtime (tests/rt/*.c -> tests/_bin/)."""
    built = None
    deps = [os.path.join(PKG, "libodp_cls.so"), os.path.join(PKG, "libodph.so"),
            os.path.join(INC, "odp_rt.h"), os.path.join(INC, "odp", "helper", "odph_api.h")]
    for name in ("rx_driver", "rt_unit"):
        src = os.path.join(ROOT, "tests", "rt", name + ".c")
        if not os.path.exists(src):
            continue
        os.makedirs(TEST_BIN, exist_ok=True)
        out = os.path.join(TEST_BIN, name)
        if not force and not _stale(out, [src] + deps):
            continue
        _run(["gcc", "-O2", "-std=gnu11", "-Wall", "-I", INC, "-o", out, src, "-L", PKG,
              "-lodph", "-lodp_cls", "-Wl,-rpath,$ORIGIN/" + os.path.relpath(PKG, TEST_BIN),
              "-lpthread"])
        built = out
    return built


REF_EXAMPLE = "/root/reference/example/classifier/odp_classifier.c"
EX_BIN = os.path.join(ROOT, "examples", "_bin")


def build_example(force: bool = False):
    """Compile the reference's example/classifier source, unchanged, against
    this build's odp_api.h / odph_api.h and link it with libodp_cls.so +
    libodph.so (north-star acceptance: the example links and runs unchanged).
    Skipped when the reference tree is absent (GPU box: the binary travels)."""
    if not os.path.exists(REF_EXAMPLE):
        return None
    os.makedirs(EX_BIN, exist_ok=True)
    out = os.path.join(EX_BIN, "odp_classifier")
    libs = [os.path.join(PKG, "libodp_cls.so"), os.path.join(PKG, "libodph.so")]
    if not force and not _stale(out, [REF_EXAMPLE] + libs):
        return None
    _run(["gcc", "-O2", "-std=gnu11", "-I", INC, "-o", out, REF_EXAMPLE, "-L", PKG,
          "-lodph", "-lodp_cls", "-Wl,-rpath,$ORIGIN/" + os.path.relpath(PKG, EX_BIN),
          "-lpthread"])
    return out


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 2:   # python -m odp_amd._build OUT_DIR DEF=1 ...
        print(build(force=True, out_dir=sys.argv[1], defines=sys.argv[2:]))
    else:
        print(build(force=True))
