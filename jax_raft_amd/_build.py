"""In-tree native build: hipcc --offload-arch=gfx950 -> jax_raft_amd/_C.so.

No hipify, no torch JIT cache: every ``.hip`` kernel TU is compiled directly
for gfx950 and linked with the TORCH_LIBRARY binding / plan runtime into one
shared object that lives next to this file (so it ships with the repository
snapshot to the GPU box and is visibly the library the tests load).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
SO_PATH = PKG_DIR / "_C.so"
ARCH = os.environ.get("JR_OFFLOAD_ARCH") or "gfx950"   # (documented in knobs.py; _build imports nothing)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")

KERNEL_SOURCES = [
    CSRC / "kernels" / "conv_igemm.hip",
    CSRC / "kernels" / "conv_fam_r.hip",
    CSRC / "kernels" / "conv_fam_rw.hip",
    CSRC / "kernels" / "conv_fam_p.hip",
    CSRC / "kernels" / "conv_fam_m32.hip",
    CSRC / "kernels" / "conv_fam_d2.hip",
    CSRC / "kernels" / "conv_fam_g.hip",
    CSRC / "kernels" / "corr.hip",
    CSRC / "kernels" / "corr_pyr.hip",
    CSRC / "kernels" / "elementwise.hip",
    CSRC / "kernels" / "conv_f32.hip",
    CSRC / "kernels" / "f32.hip",
    CSRC / "kernels" / "flowhead.hip",
    CSRC / "kernels" / "conv_direct.hip",
    CSRC / "kernels" / "train.hip",
    CSRC / "kernels" / "wgrad.hip",
    CSRC / "kernels" / "convex_head.hip",
    CSRC / "kernels" / "conv1x1.hip",
    CSRC / "kernels" / "gru_fused.hip",
    CSRC / "kernels" / "gru_halo.hip",
    CSRC / "kernels" / "conv_halo.hip",
    CSRC / "kernels" / "bgemm.hip",
    CSRC / "kernels" / "merged.hip",
    CSRC / "kernels" / "conv_fam_grp.hip",
]
HOST_SOURCES = [CSRC / "runtime" / "binding.cpp"]
# every header of csrc/ is a dependency of every object (a missed header left stale objects in
# _C.so before: conv1x1.h, round 3); the set is small, so a rebuild on any header edit is cheap
HEADERS = sorted(CSRC.rglob("*.h"))


def _torch_paths():
    import torch
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    deps = [src] + HEADERS
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(map(str, cmd)) + "\n" + r.stdout)
    return r.stdout


SAN_BUILD = REPO / "build" / "native_san"
SAN_SO_PATH = PKG_DIR / "_C_san.so"


def build(force: bool = False, verbose: bool = False, jobs: int | None = None, sanitize: bool = False) -> Path:
    """Compile all kernels + runtime for gfx950 and link ``_C.so``.

    ``sanitize=True`` (``python -m jax_raft_amd._build --sanitize``) links
    ``_C_san.so`` instead: the same kernel objects, the host runtime (plan
    executor, graph capture / node copy, bindings) built with UndefinedBehavior
    + bounds sanitizers (host code only -- no GPU sanitizer runs on this pool).
    Load it with ``JR_NATIVE_SO=jax_raft_amd/_C_san.so`` (scripts/gpu_sanitize.sh)."""
    BUILD.mkdir(parents=True, exist_ok=True)
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    host_dir, so_path, host_flags = BUILD, SO_PATH, []
    if sanitize:
        SAN_BUILD.mkdir(parents=True, exist_ok=True)
        host_dir, so_path = SAN_BUILD, SAN_SO_PATH
        host_flags = ["-fsanitize=undefined,bounds", "-fno-sanitize=vptr", "-fno-omit-frame-pointer", "-g"]
    jobs = jobs or min(8, os.cpu_count() or 4)
    cmds = []
    objs = []
    for src in KERNEL_SOURCES:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, src):
            cmds.append([HIPCC, f"--offload-arch={ARCH}", *common, "-c", str(src), "-o", str(obj)])
    for src in HOST_SOURCES:
        obj = host_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, src):
            incs = [f"-I{p}" for p in inc] + [f"-I{py_inc}"]
            cmds.append([CXX, *common, *host_flags, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                         "-DTORCH_API_INCLUDE_EXTENSION_H", *incs, "-I/opt/rocm/include", "-c", str(src), "-o", str(obj)])
    if cmds:
        with cf.ThreadPoolExecutor(jobs) as ex:
            for out in ex.map(_run, cmds):
                if verbose and out.strip():
                    print(out)
    need_link = force or not so_path.exists() or any(o.stat().st_mtime > so_path.stat().st_mtime for o in objs)
    if need_link:
        tmp = so_path.with_suffix(".so.tmp")
        link = [
            HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp),
            f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            f"-Wl,-rpath,{lib}", "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib",
        ]
        if sanitize:   # the g++-instrumented host objects need GCC's UBSan runtime as a dependency
            ubsan = subprocess.run([CXX, "-print-file-name=libubsan.so"], stdout=subprocess.PIPE, text=True).stdout
            link.append(os.path.realpath(ubsan.strip()))
        _run(link)
        os.replace(tmp, so_path)
    return so_path


if __name__ == "__main__":
    p = build(force="--force" in sys.argv, verbose=True, sanitize="--sanitize" in sys.argv)
    print(p)
