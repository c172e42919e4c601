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
        _install(so, os.path.join(NATIVE_DIR, os.path.basename(so)))
    for exe in ("spfft_bench", "spfft_native_tests", "spfft_mpi_tests", "example_c",
                "example_cpp", "example_f90"):
        src = os.path.join(BUILD_DIR, exe)
        if os.path.exists(src):
            _install(src, os.path.join(NATIVE_DIR, exe))
    return NATIVE_DIR


def _install(src, dst):
    """Copy then rename: a process that has the old library mapped keeps its
    (unlinked) file; copying over it in place would change the pages under it."""
    tmp = dst + ".tmp"
    shutil.copy2(src, tmp)
    os.replace(tmp, dst)


def _check_targets():
    """Every kernel object must carry a gfx950 code object (and nothing else)."""
    objs = glob.glob(os.path.join(BUILD_DIR, "CMakeFiles", "spfft_amd_kernels.dir", "src", "kernels", "*.o"))
    if not objs:
        raise RuntimeError("no kernel objects found under CMakeFiles/spfft_amd_kernels.dir")
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
    _check_kernel_resources(objs)


# Stage kernels must not spill: a spill to scratch (private memory) in a stage
# kernel costs far more than its HBM traffic. The gate fails the build when a
# change makes a kernel spill. Round 2 found such a regression by profiling: a
# second FFT call site put 188 B of scratch into the run-time-engine y stage.
# The report lists VGPRs / scratch of every kernel in build/kernel_resources.txt.


def _check_kernel_resources(objs):
    llvm = os.path.join(ROCM, "llvm", "bin")
    rows, bad = [], []
    for o in sorted(objs):
        fat, co = o + ".fatbin", o + ".gfx950.co"
        try:
            subprocess.run([os.path.join(llvm, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, o],
                           check=True)
            subprocess.run([os.path.join(llvm, "clang-offload-bundler"), "--unbundle", "--type=o",
                            "--input=" + fat, "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            "--output=" + co], check=True)
            notes = subprocess.run([os.path.join(llvm, "llvm-readelf"), "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
        finally:
            for f in (fat, co):
                if os.path.exists(f):
                    os.remove(f)
        name, meta = None, {}

        def flush():
            if name is None:
                return
            rows.append((name, meta.get("vgpr_count", "?"), meta.get("private_segment_fixed_size", "?"),
                         meta.get("vgpr_spill_count", "?"), meta.get("sgpr_spill_count", "?")))
            # a few bytes of stack (a small struct) are tolerated; register
            # spills and real scratch traffic are not
            spills = (int(meta.get("vgpr_spill_count", "0")) > 0 or
                      int(meta.get("private_segment_fixed_size", "0")) > 64)
            if spills:
                bad.append(rows[-1])

        for line in notes.splitlines():
            t = line.strip()
            if t.startswith(".name:"):
                flush()
                name, meta = t.split(":", 1)[1].strip(), {}
            elif t.startswith((".vgpr_count:", ".private_segment_fixed_size:", ".vgpr_spill_count:",
                               ".sgpr_spill_count:")):
                k, v = t[1:].split(":", 1)
                meta[k] = v.strip()
        flush()
    with open(os.path.join(BUILD_DIR, "kernel_resources.txt"), "w") as f:
        f.write("kernel\tvgprs\tscratch_bytes_per_lane\tvgpr_spills\tsgpr_spills\n")
        for r in rows:
            f.write("\t".join(str(x) for x in r) + "\n")
    if bad:
        raise RuntimeError("stage kernels spill to scratch: " +
                           "; ".join(f"{r[0][:80]} (vgprs {r[1]}, scratch {r[2]} B)" for r in bad[:5]))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args(argv)
    build(a.clean, a.jobs, "Debug" if a.debug else "Release")


if __name__ == "__main__":
    sys.exit(main())
