"""In-tree build of the two native extensions of codename_symbiont_amd.

* ``codename_symbiont_amd/_hip*.so``    -- CDNA4 HIP kernels + encoder runtime, hipcc --offload-arch=gfx950
* ``codename_symbiont_amd/_native*.so`` -- host-side C++ cores (wire codec, NATS protocol, tokenizer,
                                            sentence splitter, HTML extractor, Markov, PackStream)

Both are plain ``hipcc``/``g++`` invocations (no hipify, no torch JIT cache) so the built ``.so``
files live in the source tree and travel with the repository snapshot to the GPU box.  Builds are
incremental (object mtime vs. source + header mtimes) and parallel.

Usage:  python csrc/build.py [--hip-only|--native-only] [--force] [-j N]

A/B builds of the kernels: SYMB_HIP_CXXFLAGS adds flags to every .hip compile and SYMB_BUILD_TAG
names a separate object directory and output ``_hip_<tag>.so`` (loaded instead of ``_hip`` when
SYMB_HIP_SO points at it, ops/_ext.py).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = ROOT / "codename_symbiont_amd"
BUILD = ROOT / "build"
ARCH = os.environ.get("SYMB_OFFLOAD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.environ.get("HIPCC", f"{ROCM}/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _py_include() -> str:
    return sysconfig.get_paths()["include"]


def _newest(paths) -> float:
    return max((p.stat().st_mtime for p in paths if p.exists()), default=0.0)


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + proc.stdout + proc.stderr)
        raise RuntimeError(f"compile failed: {cmd[-1] if cmd else cmd}")


def _compile_all(jobs: list[tuple[list[str], Path, Path, float]], nproc: int, force: bool) -> bool:
    todo = []
    for cmd, src, obj, dep_mtime in jobs:
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, dep_mtime):
            todo.append(cmd)
    if todo:
        with ThreadPoolExecutor(max_workers=max(1, nproc)) as ex:
            list(ex.map(_run, todo))
    return bool(todo)


# per-file code-generation flags.  The stream scans keep their MFMA accumulators in VGPRs
# (`-amdgpu-mfma-vgpr-form`): the default AGPR form copied operands and results through
# v_accvgpr moves in the hot loop -- 100M x 384 int8 scan 11.36 -> 10.94 ms, MX-fp4 5.59 -> 5.05,
# MX-fp6 7.26 -> 6.67 (profiles/r5_scan/ab_vgpr_form.jsonl)
FILE_FLAGS = {"index_stream.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def build_hip(force: bool = False, nproc: int = 8) -> Path:
    src_dir = CSRC / "hip"
    tag = os.environ.get("SYMB_BUILD_TAG", "")
    obj_dir = BUILD / ("hip_" + tag if tag else "hip")
    obj_dir.mkdir(parents=True, exist_ok=True)
    headers = list(src_dir.glob("*.h"))
    hdr_mtime = _newest(headers)
    common = [
        HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
        "-Wno-unused-result", f"-I{src_dir}", *os.environ.get("SYMB_HIP_CXXFLAGS", "").split(),
    ]
    jobs = []
    objs = []
    for src in sorted(src_dir.glob("*.hip")):
        obj = obj_dir / (src.stem + ".o")
        jobs.append((common + FILE_FLAGS.get(src.name, []) + ["-c", str(src), "-o", str(obj)], src,
                     obj, max(hdr_mtime, Path(__file__).stat().st_mtime)))
        objs.append(obj)
    # host-only C++ (the hipBLASLt plan cache for the plain projections)
    lt = src_dir / "gemm_lt.cpp"
    lt_obj = obj_dir / "gemm_lt.o"
    jobs.append(([HIPCC, "-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"-I{src_dir}",
                  "-D__HIP_PLATFORM_AMD__", "-c", str(lt), "-o", str(lt_obj)], lt, lt_obj, hdr_mtime))
    objs.append(lt_obj)
    bind = src_dir / "bindings.cpp"
    bind_obj = obj_dir / "bindings.o"
    jobs.append(
        (
            [HIPCC, "-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"-I{src_dir}",
             f"-I{_pybind_include()}", f"-I{_py_include()}", "-D__HIP_PLATFORM_AMD__",
             "-c", str(bind), "-o", str(bind_obj)],
            bind, bind_obj, hdr_mtime,
        )
    )
    objs.append(bind_obj)
    changed = _compile_all(jobs, nproc, force)
    out = PKG / (f"_hip_{tag}.so" if tag else f"_hip{EXT_SUFFIX}")
    if changed or force or not out.exists() or out.stat().st_mtime < _newest(objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs),
              f"-L{ROCM}/lib", "-lhipblaslt", f"-Wl,-rpath,{ROCM}/lib", "-o", str(out)])
    return out


def build_native(force: bool = False, nproc: int = 8) -> Path:
    src_dir = CSRC / "native"
    obj_dir = BUILD / "native"
    obj_dir.mkdir(parents=True, exist_ok=True)
    headers = list(src_dir.glob("*.h"))
    hdr_mtime = _newest(headers)
    extra = os.environ.get("SYMB_NATIVE_CXXFLAGS", "").split()
    common = [
        CXX, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"-I{src_dir}",
        f"-I{_pybind_include()}", f"-I{_py_include()}", *extra,
    ]
    jobs, objs = [], []
    for src in sorted(src_dir.glob("*.cpp")):
        obj = obj_dir / (src.stem + ".o")
        jobs.append((common + ["-c", str(src), "-o", str(obj)], src, obj, hdr_mtime))
        objs.append(obj)
    changed = _compile_all(jobs, nproc, force)
    out = PKG / f"_native{EXT_SUFFIX}"
    if changed or force or not out.exists() or out.stat().st_mtime < _newest(objs):
        _run([CXX, "-shared", "-fPIC", *extra, *map(str, objs), "-o", str(out)])
    return out


def build_all(force: bool = False, nproc: int | None = None, hip: bool = True, native: bool = True):
    nproc = nproc or min(8, os.cpu_count() or 4)
    outs = []
    if native and list((CSRC / "native").glob("*.cpp")):
        outs.append(build_native(force, nproc))
    if hip:
        outs.append(build_hip(force, nproc))
    return outs


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hip-only", action="store_true")
    ap.add_argument("--native-only", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    outs = build_all(a.force, a.j, hip=not a.native_only, native=not a.hip_only)
    for o in outs:
        print(o)


if __name__ == "__main__":
    main()
