"""Host sanitizer runs (race detection / sanitizers).

Builds the library, the native test runner, the C++ example and the benchmark
CLI with host-only sanitizers (CMake SPFFT_SANITIZE; device code unchanged) in
build/san-<kind>/ and runs the host (SPFFT_PU_HOST) paths under them:

  * asan: AddressSanitizer + UndefinedBehaviorSanitizer (buffer overruns in
    the index plan, compression, host FFT and exchange layouts; UB in the
    64-bit offset arithmetic);
  * tsan: ThreadSanitizer (the host executor's thread pool, in-process rank
    groups exchanging through the local communicator, timing tree).

    python tools/sanitize.py asan|tsan [--jobs N]

Exit status 0 when every program ran clean. CPU only: GPU sanitizers and
xnack-enabled code objects are not used.
"""
import argparse
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
KINDS = {"asan": "address,undefined", "tsan": "thread"}


def build(kind, jobs):
    bdir = os.path.join(REPO, "build", f"san-{kind}")
    clang = os.path.join(ROCM, "llvm", "bin")
    if not os.path.exists(os.path.join(bdir, "build.ninja")):
        subprocess.run(["cmake", "-S", REPO, "-B", bdir, "-G", "Ninja", "-DCMAKE_BUILD_TYPE=RelWithDebInfo",
                        f"-DCMAKE_C_COMPILER={clang}/clang", f"-DCMAKE_CXX_COMPILER={clang}/clang++",
                        f"-DCMAKE_HIP_COMPILER={clang}/clang++", "-DCMAKE_HIP_ARCHITECTURES=gfx950",
                        # kernels without debug info: they are not sanitized, and -g
                        # multiplies their compile time
                        "-DCMAKE_HIP_FLAGS_RELWITHDEBINFO=-O3 -DNDEBUG",
                        f"-DSPFFT_SANITIZE={KINDS[kind]}", "-DSPFFT_MPI=OFF", "-DSPFFT_FORTRAN=OFF"],
                       check=True, stdout=subprocess.DEVNULL)
    subprocess.run(["cmake", "--build", bdir, "-j", str(jobs), "--target", "spfft_native_tests",
                    "example_cpp", "example_c", "spfft_bench"], check=True, stdout=subprocess.DEVNULL)
    return bdir


def run(kind, bdir):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=0:detect_odr_violation=0:abort_on_error=0:halt_on_error=1:exitcode=86"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1:exitcode=87"
    env["TSAN_OPTIONS"] = "halt_on_error=1:exitcode=88:report_signal_unsafe=0"
    env["HIP_VISIBLE_DEVICES"] = env.get("SPFFT_SAN_DEVICES", "")  # host paths only
    env["OMP_NUM_THREADS"] = "4"
    progs = [
        [os.path.join(bdir, "spfft_native_tests")],
        [os.path.join(bdir, "example_cpp")],
        [os.path.join(bdir, "example_c")],
        [os.path.join(bdir, "spfft_bench"), "-d", "24", "20", "18", "-r", "2", "-o",
         os.path.join(bdir, "bench.json"), "-e", "all", "-p", "cpu", "-m", "2", "--cutoff", "0.5"],
    ]
    ok = True
    for cmd in progs:
        r = subprocess.run(cmd, cwd=bdir, env=env, capture_output=True, text=True, timeout=900)
        out = r.stdout + r.stderr
        bad = r.returncode != 0 or "Sanitizer" in out or "runtime error:" in out
        print(f"[{kind}] {os.path.basename(cmd[0])}: rc={r.returncode} {'FAIL' if bad else 'clean'}")
        if bad:
            ok = False
            print(out[-6000:])
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=sorted(KINDS))
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args()
    bdir = build(a.kind, a.jobs)
    sys.exit(0 if run(a.kind, bdir) else 1)


if __name__ == "__main__":
    main()
