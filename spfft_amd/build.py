"""Builds the native library in-tree (CMake + Ninja, hipcc/clang for gfx950).

    python -m spfft_amd.build [--clean] [--jobs N]

The shared libraries are copied into spfft_amd/_native/ where the Python front
end loads them (and where a gpurun snapshot carries them to the GPU box).
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD_DIR = os.path.join(REPO, "build")
NATIVE_DIR = os.path.join(REPO, "spfft_amd", "_native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _run(cmd, **kw):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, **kw)


def build(clean: bool = False, jobs: int | None = None, build_type: str = "Release") -> str:
    if clean and os.path.isdir(BUILD_DIR):
        shutil.rmtree(BUILD_DIR)
    jobs = jobs or min(16, os.cpu_count() or 4)
    env = dict(os.environ)
    env.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    clang = os.path.join(ROCM, "llvm", "bin")
    if not os.path.exists(os.path.join(BUILD_DIR, "build.ninja")):
        _run(["cmake", "-S", REPO, "-B", BUILD_DIR, "-G", "Ninja",
              f"-DCMAKE_BUILD_TYPE={build_type}",
              f"-DCMAKE_C_COMPILER={clang}/clang", f"-DCMAKE_CXX_COMPILER={clang}/clang++",
              f"-DCMAKE_HIP_COMPILER={clang}/clang++", "-DCMAKE_HIP_ARCHITECTURES=gfx950"], env=env)
    _run(["cmake", "--build", BUILD_DIR, "-j", str(jobs)], env=env)
    _check_targets()
    os.makedirs(NATIVE_DIR, exist_ok=True)
    for so in glob.glob(os.path.join(BUILD_DIR, "libspfft_amd*.so")):
        shutil.copy2(so, os.path.join(NATIVE_DIR, os.path.basename(so)))
    for exe in ("spfft_bench", "spfft_native_tests", "spfft_mpi_tests", "example_c",
                "example_cpp", "example_f90"):
        src = os.path.join(BUILD_DIR, exe)
        if os.path.exists(src):
            shutil.copy2(src, os.path.join(NATIVE_DIR, exe))
    return NATIVE_DIR


def _check_targets():
    """Every kernel object must carry a gfx950 code object (and nothing else)."""
    objs = glob.glob(os.path.join(BUILD_DIR, "CMakeFiles", "spfft_amd.dir", "src", "kernels", "*.o"))
    llvm = os.path.join(ROCM, "llvm", "bin")
    for o in objs:
        tmp = o + ".fatbin"
        subprocess.run([os.path.join(llvm, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + tmp, o],
                       check=True)
        out = subprocess.run([os.path.join(llvm, "clang-offload-bundler"), "--list", "--type=o",
                              "--input=" + tmp], check=True, capture_output=True, text=True).stdout
        os.remove(tmp)
        gpus = [l for l in out.split() if "amdgcn" in l]
        if not gpus or any(not l.endswith("gfx950") for l in gpus):
            raise RuntimeError(f"{o}: unexpected offload targets {gpus}")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args(argv)
    build(a.clean, a.jobs, "Debug" if a.debug else "Release")


if __name__ == "__main__":
    sys.exit(main())
