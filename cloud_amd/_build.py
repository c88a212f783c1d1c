"""In-tree native build for cloud_amd (gfx950 HIP kernels + C++ runtime pieces).

Two shared objects are produced next to this file:

* ``_C<EXT_SUFFIX>``      -- HIP/CDNA4 kernels (``csrc/kernels/*.hip``) + pybind11
  bindings (``csrc/bindings.cpp``).  Linked against ``libamdhip64.so.7``; at run
  time the SONAME resolves to the HIP runtime that ``import torch`` already
  mapped, so exactly one HIP runtime lives in the process.
* ``_comm<EXT_SUFFIX>``     -- native RCCL communicator (``csrc/comm/rccl_comm.cpp``):
  collectives on a side HIP stream for the bucketed DP engine.  Linked against
  ``librccl.so.1``, which resolves to the RCCL ``import torch`` already mapped.
* ``_data<EXT_SUFFIX>``     -- native input pipeline (``csrc/data/loader.cpp``): mmap'd
  .npy arrays, shuffled / rank-sharded batches gathered by C++ worker threads into
  pinned slot buffers; host-only.
* ``_monitoring<EXT_SUFFIX>`` -- the C++ metrics registry / periodic exporter
  (``csrc/monitoring/*.cpp``), host-only, no HIP dependency, so CPU boxes can use
  it (parity target: reference ``src/cpp/monitoring/*``).

No hipify, no torch C++ headers: kernels take raw device pointers and a
``hipStream_t`` handed over from ``torch.cuda.current_stream().cuda_stream``.
Objects are cached by a content hash of (source, flags) under ``build/``.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "cloud_amd"
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("CLOUD_AMD_ARCH", "gfx950")

HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
    "-munsafe-fp-atomics", "-ffp-contract=fast",
    "-Wno-unused-result", "-Wno-unused-command-line-argument",
]
CXX_FLAGS = ["-O2", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function"]


def _py_includes():
    import pybind11  # noqa: WPS433

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _hipcc():
    p = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    if not Path(p).exists():
        raise RuntimeError("hipcc not found; cloud_amd needs ROCm to build its gfx950 kernels")
    return p


def _digest(src: Path, flags) -> str:
    h = hashlib.sha1()
    h.update(src.read_bytes())
    for inc in sorted((CSRC / "include").glob("*.h")) + sorted(src.parent.glob("*.h")):
        h.update(inc.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _compile(compiler, src: Path, flags, verbose=False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    obj = BUILD / f"{src.stem}.{_digest(src, flags)}.o"
    if obj.exists():
        return obj
    cmd = [compiler, *flags, "-c", str(src), "-o", str(obj) + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    os.replace(str(obj) + ".tmp", obj)
    return obj


def _link(compiler, objs, out: Path, extra, verbose=False):
    tmp = out.with_suffix(out.suffix + ".tmp")
    cmd = [compiler, "-shared", "-fPIC", *map(str, objs), "-o", str(tmp), *extra]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {out}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)


def kernel_sources():
    return sorted((CSRC / "kernels").glob("*.hip"))


def experimental_flags():
    """CLOUD_AMD_BUILD_EXPERIMENTAL=1 compiles the experiment-only GEMM cores (glds8, the
    256 x 256 ring core, stream-K, 256 x 128) into _C for A/B runs; the default build leaves
    them out."""
    return ["-DCA_EXPERIMENTAL=1"] if os.environ.get("CLOUD_AMD_BUILD_EXPERIMENTAL") == "1" else []


def build_kernels(verbose=False, jobs=None) -> Path:
    hipcc = _hipcc()
    inc = [f"-I{CSRC / 'include'}"] + experimental_flags()
    srcs = kernel_sources()
    bind = CSRC / "bindings.cpp"
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, hipcc, s, HIP_FLAGS + inc, verbose) for s in srcs]
        futs.append(ex.submit(_compile, hipcc, bind, HIP_FLAGS + inc + _py_includes(), verbose))
        objs = [f.result() for f in futs]
    out = PKG / f"_C{EXT_SUFFIX}"
    _link(hipcc, objs, out, [f"--offload-arch={ARCH}", f"-L{ROCM / 'lib'}", "-lamdhip64"], verbose)
    return out


def build_comm(verbose=False) -> Path:
    hipcc = _hipcc()
    src = CSRC / "comm" / "rccl_comm.cpp"
    flags = ["-O2", "-fPIC", "-std=c++17", f"-I{ROCM / 'include'}", "-Wno-unused-command-line-argument"]
    obj = _compile(hipcc, src, flags + _py_includes(), verbose)
    out = PKG / f"_comm{EXT_SUFFIX}"
    _link(hipcc, [obj], out, [f"-L{ROCM / 'lib'}", "-lrccl", "-lamdhip64"], verbose)
    return out


def build_monitoring(verbose=False) -> Path:
    cxx = shutil.which("g++") or "c++"
    inc = [f"-I{CSRC / 'include'}", f"-I{CSRC / 'monitoring'}"]
    srcs = sorted((CSRC / "monitoring").glob("*.cpp"))
    srcs = [s for s in srcs if not s.name.endswith("_test.cpp")]
    objs = [_compile(cxx, s, CXX_FLAGS + inc + _py_includes(), verbose) for s in srcs]
    out = PKG / f"_monitoring{EXT_SUFFIX}"
    _link(cxx, objs, out, ["-lpthread"], verbose)
    return out


def build_data(verbose=False) -> Path:
    cxx = shutil.which("g++") or "c++"
    src = CSRC / "data" / "loader.cpp"
    obj = _compile(cxx, src, CXX_FLAGS + _py_includes(), verbose)
    out = PKG / f"_data{EXT_SUFFIX}"
    _link(cxx, [obj], out, ["-lpthread"], verbose)
    return out


def build_loader_test(sanitize=None, verbose=False) -> Path:
    """Standalone multi-threaded test of the input-pipeline core (csrc/data/loader_core.h,
    no Python).  ``sanitize``: None, "address" (ASan+UBSan) or "thread" (TSan)."""
    cxx = shutil.which("g++") or "c++"
    src = CSRC / "data" / "loader_test.cpp"
    tag = {None: "", "address": "_asan", "thread": "_tsan"}[sanitize]
    out = BUILD / f"loader_test{tag}"
    BUILD.mkdir(parents=True, exist_ok=True)
    flags = ["-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-I{CSRC / 'data'}"]
    if sanitize == "address":
        flags += ["-fsanitize=address,undefined"]
    elif sanitize == "thread":
        flags += ["-fsanitize=thread"]
    cmd = [cxx, *flags, str(src), "-o", str(out), "-lpthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {src}\n{r.stdout}\n{r.stderr}")
    return out


def build_monitoring_test(verbose=False) -> Path:
    """Standalone C++ golden-test binary for the metrics library (no Python)."""
    cxx = shutil.which("g++") or "c++"
    inc = [f"-I{CSRC / 'include'}", f"-I{CSRC / 'monitoring'}"]
    lib_srcs = [s for s in sorted((CSRC / "monitoring").glob("*.cpp"))
                if s.name not in ("bindings_monitoring.cpp",) and not s.name.endswith("_test.cpp")]
    test_src = CSRC / "monitoring" / "monitoring_test.cpp"
    out = BUILD / "monitoring_test"
    BUILD.mkdir(parents=True, exist_ok=True)
    cmd = [cxx, *CXX_FLAGS, *inc, *map(str, lib_srcs), str(test_src), "-o", str(out), "-lpthread"]
    if os.environ.get("CLOUD_AMD_SANITIZE"):
        cmd[1:1] = ["-fsanitize=address,undefined", "-g"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"monitoring test build failed\n{r.stdout}\n{r.stderr}")
    return out


def build_gemm_bench(verbose=False) -> Path:
    """bin/gemm_bench: the standalone GEMM-core benchmark + fp32-reference check
    (csrc/tests/gemm_bench.hip; no Python on the GPU side)."""
    out = PKG.parent / "bin" / "gemm_bench"
    out.parent.mkdir(parents=True, exist_ok=True)
    cmd = [_hipcc(), *[f for f in HIP_FLAGS if f != "-fPIC"], f"-I{CSRC / 'include'}",
           str(CSRC / "tests" / "gemm_bench.hip"), "-o", str(out)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"gemm_bench build failed\n{r.stdout}\n{r.stderr}")
    return out


def build_all(verbose=False):
    outs = [build_kernels(verbose)]
    if (CSRC / "comm" / "rccl_comm.cpp").exists():
        outs.append(build_comm(verbose))
    if (CSRC / "monitoring").exists() and any((CSRC / "monitoring").glob("*.cpp")):
        outs.append(build_monitoring(verbose))
    if (CSRC / "data" / "loader.cpp").exists():
        outs.append(build_data(verbose))
    return outs


if __name__ == "__main__":
    if "gemm_bench" in sys.argv:
        print(build_gemm_bench(verbose="-v" in sys.argv))
    else:
        for p in build_all(verbose="-v" in sys.argv):
            print(p)
