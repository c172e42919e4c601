"""Cache-policy audit of the built library's gfx950 kernels: counts the global
loads and stores of each kernel and how many carry the non-temporal (`nt`) bit.

Why: a run-time choice between a plain and a streaming access
(`if (plain) *p = v; else st_stream(p, v);`) is merged by the compiler into one
plain access, dropping the hint without a diagnostic (profiles/r6/ntmerge). The
stage kernels therefore take such choices as template parameters, and
tests/test_build.py::test_stage_kernels_keep_nt_hints checks the result here.

    python tools/nt_audit.py [library.so] [kernel-name-regex]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _tool(name):
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    p = os.path.join(rocm, "llvm", "bin", name)
    return p if os.path.exists(p) else shutil.which(name)


def code_objects(lib, workdir):
    """Paths of the gfx950 code objects in the library's .hip_fatbin section
    (one offload bundle per translation unit, concatenated)."""
    fat = os.path.join(workdir, "fat.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    bundler = _tool("clang-offload-bundler")
    for i, o in enumerate(offs):
        end = offs[i + 1] if i + 1 < len(offs) else len(data)
        piece = os.path.join(workdir, f"b{i}.bin")
        with open(piece, "wb") as f:
            f.write(data[o:end])
        co = os.path.join(workdir, f"b{i}.co")
        r = subprocess.run([bundler, "-type=o", f"-targets={TARGET}", f"-input={piece}", f"-output={co}",
                            "-unbundle"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def audit(lib, pattern=r".*", needles=()):
    """{kernel symbol: dict(st, st_nt, ld, ld_nt)} for the kernels matching pattern
    (only code objects that contain one of the byte strings `needles`, if given,
    are disassembled)."""
    rx = re.compile(pattern)
    res = {}
    objdump = _tool("llvm-objdump")
    with tempfile.TemporaryDirectory() as wd:
        for co in code_objects(lib, wd):
            if needles:
                blob = open(co, "rb").read()
                if not any(n in blob for n in needles):
                    continue
            txt = subprocess.run([objdump, "-d", "--no-show-raw-insn", co], capture_output=True, text=True,
                                 check=True).stdout
            name, counts = None, None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if m:
                    name = m.group(1)
                    counts = res.setdefault(name, dict(st=0, st_nt=0, ld=0, ld_nt=0)) if rx.search(name) else None
                    continue
                if counts is None:
                    continue
                ins = line.strip()
                kind = "st" if re.match(r"(global|buffer)_store", ins) else (
                    "ld" if re.match(r"(global|buffer)_load", ins) else None)
                if kind:
                    counts[kind] += 1
                    if re.search(r"\bnt\b", ins):
                        counts[kind + "_nt"] += 1
    return res


if __name__ == "__main__":
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(repo, "spfft_amd", "_native", "libspfft_amd.so")
    pat = sys.argv[2] if len(sys.argv) > 2 else r"(z|y)_(backward|forward)"
    for k, c in sorted(audit(lib, pat).items()):
        print(f"{c['st']:4d} st {c['st_nt']:4d} nt | {c['ld']:4d} ld {c['ld_nt']:4d} nt  {k}")
