"""In-tree build of the package's native extensions for gfx950 (MI355X).

The HIP kernels are compiled with ``hipcc --offload-arch=gfx950`` directly (no
hipify step, no torch JIT cache): the resulting ``.so`` files live next to the
Python sources so they travel with the repository snapshot to the GPU box.

Extensions
----------
``_C``      torch binding of the compute kernels (csrc/*.hip + csrc/bindings.cpp)
``_comm``   C++ communication engine (csrc/comm/*): RCCL communicator, xGMI
            IPC peer buffers and one-shot allreduce, Horovod-style fusion engine.

Usage: ``python -m ray_lightning_accelerators_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import Dict, List, Sequence

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR.parent / "build" / "native"
ARCH = os.environ.get("RLA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths() -> Dict[str, object]:
    import torch
    import torch.utils.cpp_extension as ce

    tdir = Path(torch.__file__).resolve().parent
    return {
        "includes": [str(tdir / "include"), str(tdir / "include/torch/csrc/api/include")],
        "libdir": str(tdir / "lib"),
        "abi": int(torch._C._GLIBCXX_USE_CXX11_ABI),
        "pyinc": sysconfig.get_paths()["include"],
    }


EXTENSIONS = {
    "_C": {
        "hip": ["optim_kernels.hip", "mlp_kernels.hip", "mlp_adam.hip", "mlp_step3.hip", "bn_act.hip", "pool.hip", "conv_wgrad.hip", "conv3x3.hip", "conv1x1.hip", "stem.hip"],
        "cpp": ["bindings.cpp"],
        "torch": True,
        "libs": [],
    },
    "_comm": {
        "hip": ["comm/xgmi_allreduce.hip", "comm/xgmi_twoshot.hip", "comm/pack.hip"],
        "cpp": ["comm/comm_bindings.cpp", "comm/communicator.cpp", "comm/fusion_engine.cpp", "comm/reducer.cpp"],
        "torch": True,
        "libs": ["rccl"],
    },
}


def ext_path(name: str) -> Path:
    return PKG_DIR / f"{name}{sysconfig.get_config_var('EXT_SUFFIX')}"


def _headers() -> List[Path]:
    return list(CSRC.rglob("*.h"))


def _needs_build(target: Path, sources: Sequence[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(s.stat().st_mtime > t for s in list(sources) + _headers())


def _run(cmd: List[str]) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        sys.stderr.write(proc.stdout)
        raise RuntimeError(f"native build step failed ({proc.returncode}): {' '.join(cmd[:4])} ...")


def build_extension(name: str, force: bool = False, jobs: int = 4, verbose: bool = False) -> Path:
    spec = EXTENSIONS[name]
    target = ext_path(name)
    hip_srcs = [CSRC / s for s in spec["hip"]]
    cpp_srcs = [CSRC / s for s in spec["cpp"]]
    missing = [str(s) for s in hip_srcs + cpp_srcs if not s.exists()]
    if missing:
        raise FileNotFoundError(f"missing sources for {name}: {missing}")
    if not force and not _needs_build(target, hip_srcs + cpp_srcs):
        return target
    tp = _torch_paths()
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    common = [
        "-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", f"-I{tp['pyinc']}",
        f"-D_GLIBCXX_USE_CXX11_ABI={tp['abi']}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
        f"-DTORCH_EXTENSION_NAME={name}", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-unused-result", "-Wno-deprecated-declarations",
    ]
    tinc = [f"-I{p}" for p in tp["includes"]]
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = BUILD_DIR / f"{name}__{src.stem}.o"
        objs.append(obj)
        jobs_list.append([HIPCC, "-x", "hip", f"--offload-arch={ARCH}", *common, "-c", str(src), "-o", str(obj)])
    for src in cpp_srcs:
        obj = BUILD_DIR / f"{name}__{src.stem}.o"
        objs.append(obj)
        jobs_list.append([HIPCC, *common, *tinc, "-c", str(src), "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, c) for c in jobs_list]:
            f.result()
    libdir = tp["libdir"]
    # Link with the host compiler against torch's OWN HIP runtime / RCCL (they
    # carry no SONAME, so the NEEDED entries resolve to the copies torch has
    # already loaded -- never a second HIP runtime from /opt/rocm).
    link = ["g++", "-shared", "-fPIC", *map(str, objs), "-o", str(target) + ".tmp",
            f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-ltorch", "-ltorch_cpu",
            "-ltorch_python", "-lc10_hip", "-ltorch_hip", "-lamdhip64"]
    for lib in spec["libs"]:
        link.append(f"-l{lib}")
    _run(link)
    os.replace(str(target) + ".tmp", target)
    if verbose:
        print(f"built {target}")
    return target


SELFTEST_SOURCES = ["comm/selftest.cpp", "comm/communicator.cpp", "comm/fusion_engine.cpp", "comm/reducer.cpp",
                    "comm/xgmi_allreduce.hip", "comm/xgmi_twoshot.hip", "comm/pack.hip"]
# host-only sanitizers: each -fsanitize= directly after -Xarch_host, device code untouched
SANITIZE_HOST = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                 "-Xarch_host", "-fno-omit-frame-pointer"]
CLANGXX = os.environ.get("RLA_CLANGXX", "/opt/rocm/lib/llvm/bin/clang++")


def selftest_path(sanitize: bool) -> Path:
    return BUILD_DIR.parent / ("comm_selftest_asan" if sanitize else "comm_selftest")


def build_selftest(sanitize: bool = False, force: bool = False, jobs: int = 4, verbose: bool = False) -> Path:
    """Standalone native test of the comm engine (csrc/comm/selftest.cpp): no torch,
    forks W ranks that drive the xGMI kernels, fusion engine and reducer.  The
    ``sanitize`` build instruments the HOST code with ASan + UBSan (+ LeakSanitizer)."""
    target = selftest_path(sanitize)
    srcs = [CSRC / s for s in SELFTEST_SOURCES]
    if not force and not _needs_build(target, srcs):
        return target
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    tag = "asan" if sanitize else "plain"
    flags = ["-O1" if sanitize else "-O2", "-g", "-std=c++17", f"-I{CSRC}", "-D__HIP_PLATFORM_AMD__=1"]
    if sanitize:
        flags += SANITIZE_HOST
    objs, cmds = [], []
    for src in srcs:
        obj = BUILD_DIR / f"selftest_{tag}__{src.stem}.o"
        objs.append(obj)
        # every TU as HIP: the .cpp files include hip_runtime and launch through it
        cmds.append([HIPCC, "-x", "hip", f"--offload-arch={ARCH}", *flags, "-c", str(src), "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, c) for c in cmds]:
            f.result()
    link = [CLANGXX, *map(str, objs), "-o", str(target) + ".tmp", "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib",
            "-lamdhip64", "-lrccl", "-lpthread"]
    if sanitize:
        link += ["-fsanitize=address,undefined"]
    _run(link)
    os.replace(str(target) + ".tmp", target)
    if verbose:
        print(f"built {target}")
    return target


def build_all(force: bool = False, jobs: int = 4, verbose: bool = False, names=None) -> List[Path]:
    out = []
    for name in names or EXTENSIONS:
        spec = EXTENSIONS[name]
        srcs = [CSRC / s for s in spec["hip"] + spec["cpp"]]
        if not all(s.exists() for s in srcs):
            if verbose:
                print(f"skip {name}: sources not present")
            continue
        out.append(build_extension(name, force=force, jobs=jobs, verbose=verbose))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=int(os.environ.get("MAX_JOBS", "4")))
    ap.add_argument("--selftest", action="store_true",
                    help="also build the native comm self-test (plain + host ASan/UBSan)")
    ap.add_argument("names", nargs="*")
    args = ap.parse_args(argv)
    build_all(force=args.force, jobs=min(args.jobs, 16), verbose=True, names=args.names or None)
    if args.selftest:
        for san in (False, True):
            build_selftest(sanitize=san, force=args.force, jobs=min(args.jobs, 16), verbose=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
