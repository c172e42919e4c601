"""Builds variants of libspfft_amd.so with extra compile flags into
spfft_amd/_native/variants/libspfft_amd_<name>.so; select one at run time with
SPFFT_AMD_LIBRARY=<path>. The product kernels carry no A/B switches: an
experiment is a source patch plus a variant build of it (e.g. a different
SPFFT_MR_SIZES list, the one user-facing kernel configuration).

    python tools/build_variants.py name=-DKNOB=1,-DOTHER=2 [name2=...]
"""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def build_variant(name, flags):
    bdir = os.path.join(REPO, "build", "variants", name)
    clang = os.path.join(ROCM, "llvm", "bin")
    if not os.path.exists(os.path.join(bdir, "build.ninja")):
        subprocess.run(["cmake", "-S", REPO, "-B", bdir, "-G", "Ninja", "-DCMAKE_BUILD_TYPE=Release",
                        f"-DCMAKE_C_COMPILER={clang}/clang", f"-DCMAKE_CXX_COMPILER={clang}/clang++",
                        f"-DCMAKE_HIP_COMPILER={clang}/clang++", "-DCMAKE_HIP_ARCHITECTURES=gfx950",
                        f"-DCMAKE_HIP_FLAGS={' '.join(flags)}", f"-DCMAKE_CXX_FLAGS={' '.join(flags)}"],
                       check=True, stdout=subprocess.DEVNULL)
    subprocess.run(["cmake", "--build", bdir, "--target", "spfft_amd", "-j", "16"], check=True,
                   stdout=subprocess.DEVNULL)
    out = os.path.join(REPO, "spfft_amd", "_native", "variants")
    os.makedirs(out, exist_ok=True)
    dst = os.path.join(out, f"libspfft_amd_{name}.so")
    shutil.copy2(os.path.join(bdir, "libspfft_amd.so"), dst)
    print(dst)


if __name__ == "__main__":
    for arg in sys.argv[1:]:
        name, _, fl = arg.partition("=")
        build_variant(name, [f for f in fl.split(",") if f])
