"""In-tree native build (no JIT cache, no hipify): the .so files land inside the package so they
travel with the repo snapshot to the GPU box.

  * ``ops/_hip_kernels*.so``  — gfx950 HIP kernels (csrc/kernels/*.hip) + torch bindings
                                (csrc/bindings.cpp), compiled with ``hipcc --offload-arch=gfx950``.
  * ``engine/_runtime*.so``   — C++ serving runtime (csrc/runtime/*.cpp: paged-KV block manager with
                                prefix-hash cache, scheduler core), g++ + pybind11, no GPU needed.

Usage: ``python -m distributed_llm_amd._build [--force] [--only hip|runtime]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed_llm_amd")
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

HIP_SO = os.path.join(PKG, "ops", "_hip_kernels" + EXT)
RT_SO = os.path.join(PKG, "engine", "_runtime" + EXT)


def _newer(target: str, sources: List[str]) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(s) <= t for s in sources)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def build_hip(force: bool = False, jobs: int = 8) -> str:
    kdir = os.path.join(CSRC, "kernels")
    kernels = sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".hip"))
    headers = [os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".h")]
    bind = os.path.join(CSRC, "bindings.cpp")
    if not force and _newer(HIP_SO, kernels + headers + [bind]):
        return HIP_SO
    import torch
    from torch.utils import cpp_extension as ce
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    common = ["-fPIC", "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              "-Wno-unused-result", "-Wno-deprecated-declarations"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    torch_inc = []
    for p in ce.include_paths(device_type="cuda"):
        torch_inc += ["-isystem", p]
    py_inc = ["-isystem", sysconfig.get_paths()["include"]]
    jobs_list = []
    for src in kernels:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        jobs_list.append([hipcc, *common, "-I", kdir, "-c", src, "-o", obj])
    bind_obj = os.path.join(BUILD, "bindings.o")
    jobs_list.append([hipcc, *common, *torch_inc, *py_inc, f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                      "-DTORCH_EXTENSION_NAME=_hip_kernels", "-DTORCH_API_INCLUDE_EXTENSION_H",
                      "-c", bind, "-o", bind_obj])
    objs = [j[-1] for j in jobs_list]
    # incremental: an object newer than its source and every kernel header is reused
    srcs = kernels + [bind]
    todo = [j for j, src in zip(jobs_list, srcs) if force or not _newer(j[-1], [src] + headers)]
    with cf.ThreadPoolExecutor(max(1, min(jobs, len(todo) or 1))) as ex:
        list(ex.map(_run, todo))
    libdir = ce.library_paths(device_type="cuda")[0]
    tmp = HIP_SO + ".tmp"
    _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp, "-L", libdir,
          "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
          f"-Wl,-rpath,{libdir}"])
    os.replace(tmp, HIP_SO)
    return HIP_SO


def build_runtime(force: bool = False) -> str:
    rdir = os.path.join(CSRC, "runtime")
    srcs = sorted(os.path.join(rdir, f) for f in os.listdir(rdir) if f.endswith(".cpp"))
    hdrs = [os.path.join(rdir, f) for f in os.listdir(rdir) if f.endswith(".h")]
    if not srcs:
        return ""
    if not force and _newer(RT_SO, srcs + hdrs):
        return RT_SO
    import pybind11
    cxx = os.environ.get("CXX", "g++")
    tmp = RT_SO + ".tmp"
    _run([cxx, "-O2", "-shared", "-fPIC", "-std=c++17", "-Wall", "-I", pybind11.get_include(),
          "-isystem", sysconfig.get_paths()["include"], *srcs, "-o", tmp])
    os.replace(tmp, RT_SO)
    return RT_SO


def build_all(force: bool = False) -> List[str]:
    out = [build_runtime(force)]
    out.append(build_hip(force))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["hip", "runtime"])
    a = ap.parse_args()
    if a.only == "hip":
        print(build_hip(a.force))
    elif a.only == "runtime":
        print(build_runtime(a.force))
    else:
        print("\n".join(build_all(a.force)))
    sys.exit(0)
