"""Device memory per rank of a GPU grid, and the largest cubic grid that fits one
MI355X (288 GB HBM3E), from the grid sizing rules of src/api/grid_impl.cpp:

  planeElems = maxX * (maxY + 32) * maxLocalZ          (complex elements)
  stick side = (maxZ + 32) * maxSticks                   (BUFFERED: at least P * gMaxSticks * gMaxLocalZ)
  slab side  = sum over ranks of maxSticks * maxLocalZ   (distributed only; BUFFERED likewise)
  space domain = planeElems
  y/x intermediate: min(planeElems, SPFFT_INTER_BYTES = 2 GiB)
plus the caller's frequency values (the spherical cutoff r = N/2 holds pi/6 N^3).

    python tools/memory_model.py [--gib 288] [--ranks 1,8]
"""
import argparse
import math

PAD = 32
INTER_CAP = 2 << 30


def grid_bytes(n, ranks, elem, cutoff=0.5, r2c=False):
    maxlz = math.ceil(n / ranks)
    half = 0.5 if r2c else 1.0  # R2C keeps the x >= 0 half of the sphere
    sticks = math.ceil(half * math.pi * (cutoff * n) ** 2 / ranks)  # sphere: pi r^2 sticks
    plane = n * (n + PAD) * maxlz
    buffers = (n + PAD) * sticks + plane  # stick side + space
    if ranks > 1:
        buffers += sticks * ranks * maxlz  # slab side
    total = buffers * elem + min(plane * elem, INTER_CAP)
    values = half * math.pi / 6 * (2 * cutoff) ** 3 * n ** 3 / ranks * elem
    return total, values


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=288e9 / (1 << 30))
    ap.add_argument("--ranks", default="1,8")
    a = ap.parse_args()
    cap = a.gib * (1 << 30)
    print(f"device memory per rank (GB = 1e9 bytes), capacity {cap / 1e9:.0f} GB")
    for ranks in (int(r) for r in a.ranks.split(",")):
        for label, elem, r2c in (("C2C fp64", 16, False), ("C2C fp32", 8, False),
                                 ("R2C fp64", 16, True), ("R2C fp32", 8, True)):
            # R2C grids are sized like C2C ones (complex elements; the real space
            # domain uses half of its buffer)
            rows = []
            for n in (256, 512, 1024, 2048, 3072, 4096):
                g, v = grid_bytes(n, ranks, elem, r2c=r2c)
                rows.append(f"{n}^3: {g / 1e9:7.1f} + {v / 1e9:6.1f}")
            lo, hi = 64, 16384
            while hi - lo > 1:
                mid = (lo + hi) // 2
                g, v = grid_bytes(mid, ranks, elem, r2c=r2c)
                if g + v <= cap:
                    lo = mid
                else:
                    hi = mid
            print(f"P={ranks} {label}: largest N = {lo} | grid + values: " + "; ".join(rows))


if __name__ == "__main__":
    main()
