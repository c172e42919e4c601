"""VGPRs / scratch / spills / LDS of the kernels in a build tree, demangled and
filtered: python tools/kres.py <build-dir> <regex> (e.g. 'y_(back|for)ward.*float, 512')."""
import glob
import os
import re
import subprocess
import sys

LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "llvm", "bin")


def resources(objs):
    out = {}
    for o in objs:
        fat, co = o + ".tmp.fatbin", o + ".tmp.co"
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, o], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fat,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        os.remove(fat)
        os.remove(co)
        name, meta = None, {}
        for line in notes.splitlines():
            t = line.strip()
            if t.startswith(".name:"):
                if name:
                    out[name] = meta
                name, meta = t.split(":", 1)[1].strip(), {}
            elif t.startswith((".vgpr_count:", ".private_segment_fixed_size:", ".vgpr_spill_count:",
                               ".group_segment_fixed_size:", ".agpr_count:")):
                k, v = t[1:].split(":", 1)
                meta[k] = v.strip()
        if name:
            out[name] = meta
    return out


def main():
    bdir, pat = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    objs = glob.glob(os.path.join(bdir, "CMakeFiles", "spfft_amd.dir", "src", "kernels", "*.o"))
    res = resources(objs)
    names = list(res)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    for n, d in sorted(zip(names, dem), key=lambda x: x[1]):
        short = re.sub(r"\(.*", "", d).replace("spfft::dev::", "").replace("spfft::", "")
        if pat.search(short):
            m = res[n]
            print(f"{short[:110]:110s} vgpr={m.get('vgpr_count')} agpr={m.get('agpr_count')} "
                  f"scratch={m.get('private_segment_fixed_size')} spill={m.get('vgpr_spill_count')}")


if __name__ == "__main__":
    main()
