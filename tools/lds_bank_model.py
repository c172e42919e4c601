"""LDS bank-conflict model of the line-fast FftCT engines (gfx950 banking rules of
MI355X_MICROARCH.md §LDS): LDS cycles of every LDS access of one workgroup for a
candidate line stride LS, to pick strides offline (SPFFT lf_padded_stride).

Instruction models (lane groups, banks):
  8-byte elements (complex<float>): ds_write_b64 / ds_write2_b64 / ds_read2_b64 in
    4 groups of 16 contiguous lanes, bank = (a/4) mod 32;
  16-byte elements (complex<double>): ds_write_b128 in 8 groups of 8 contiguous lanes,
    bank = (a/4) mod 32; ds_read_b128 in the 4 non-contiguous 16-lane groups, mod 64.
Cycles of a group = the largest number of distinct dword addresses on one bank.
"""
import itertools
import sys

R128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
R128 += [[l + 32 for l in g] for g in R128]


def group_cycles(addrs, eb, groups, nbanks):
    cyc = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs.get(lane)
            if a is None:
                continue
            for d in range(eb // 4):
                dw = a // 4 + d
                banks.setdefault(dw % nbanks, set()).add(dw)
        cyc += max((len(v) for v in banks.values()), default=0)
    return cyc


def access_cycles(addrs, eb, write):
    if eb == 8:
        return group_cycles(addrs, eb, [range(i, i + 16) for i in range(0, 64, 16)], 32)
    if write:
        return group_cycles(addrs, eb, [range(i, i + 8) for i in range(0, 64, 8)], 32)
    return group_cycles(addrs, eb, R128, 64)


def engine_accesses(N, E, radices, B, shift):
    """(is_write, lane -> (b, pos)) per LDS access instruction, for one wave-sized lane set."""
    TP = N // E
    NT = B * TP
    pad = lambda i: i + (i >> shift)
    out = []
    rs = [r for r in radices if r > 1]

    def lanes():
        for tid in range(NT):
            yield tid, tid % B, tid // B

    # first pass read (input staged in LDS), then exchanges, then result write
    def reads(R):
        for k in range(E // R):
            for r in range(R):
                out.append((False, {tid: (b, pad(t + k * TP + r * (N // R))) for tid, b, t in lanes()}))

    reads(rs[0])
    ns = 1
    for i in range(len(rs) - 1):
        R, RN = rs[i], rs[i + 1]
        for k in range(E // R):
            for r in range(R):
                acc = {}
                for tid, b, t in lanes():
                    j = t + k * TP
                    kk = j % ns
                    acc[tid] = (b, pad((j - kk) * R + kk + r * ns))
                out.append((True, acc))
        reads(RN)
        ns *= R
    RL = rs[-1]
    for k in range(E // RL):
        for r in range(RL):
            out.append((True, {tid: (b, pad(t + k * TP + r * (N // RL))) for tid, b, t in lanes()}))
    return out, NT


def cycles_for_stride(N, E, radices, B, eb, LS):
    shift = 5 if eb == 8 else 4
    accs, NT = engine_accesses(N, E, radices, B, shift)
    total = ideal = 0
    for w in range(NT // 64):
        for write, acc in accs:
            addrs = {tid - 64 * w: eb * (b * LS + p) for tid, (b, p) in acc.items()
                     if 64 * w <= tid < 64 * (w + 1)}
            total += access_cycles(addrs, eb, write)
            ideal += (4 if eb == 8 else (8 if write else 4))
    return total, ideal


def min_stride(N, eb):
    shift = 5 if eb == 8 else 4
    return N + ((N - 1) >> shift) + 1


def current_stride(N, B, eb):
    kmod = 32 if eb == 8 else 16
    ls = min_stride(N, eb)
    want = 1 if B >= kmod else (kmod // B) % kmod
    while ls % kmod != want:
        ls += 1
    return ls


if __name__ == "__main__":
    # (name, N, E, radices, B, element bytes) of the line-fast engines in use
    cases = [("f32 256", 256, 16, (16, 16, 1), 16, 8), ("f32 512 W", 512, 16, (16, 16, 2), 16, 8),
             ("f32 128", 128, 16, (16, 8, 1), 16, 8), ("f64 256 E8", 256, 8, (8, 8, 4), 8, 16),
             ("f64 512 W", 512, 8, (8, 8, 8), 8, 16), ("f64 128 E8", 128, 8, (8, 8, 2), 8, 16)]
    for name, N, E, rad, B, eb in cases:
        cur = current_stride(N, B, eb)
        c, ideal = cycles_for_stride(N, E, rad, B, eb, cur)
        best = min(range(min_stride(N, eb), min_stride(N, eb) + 64),
                   key=lambda ls: cycles_for_stride(N, E, rad, B, eb, ls)[0])
        cb, _ = cycles_for_stride(N, E, rad, B, eb, best)
        print(f"{name:12s} current LS={cur} ({cur % 32}) cycles={c} (ideal {ideal}) | best LS={best} "
              f"({best % 32}) cycles={cb}")
        sys.stdout.flush()


def padded_stride(n, eb):
    shift, kmod = (5, 32) if eb == 8 else (4, 16)
    return ((n + (n >> shift) + kmod - 1) // kmod) * kmod + 1


def lines_per_block(tp, line_bytes, budget, max_thr):
    b = max_thr // tp
    if b * line_bytes > budget:
        b = budget // line_bytes
    b = max(b, 1)
    if tp < 64:
        q = 64 // tp
        b = max((b // q) * q, q)
    return b


def lf_lines(b):
    p = 1
    while p * 2 <= b and p * 2 <= 16:
        p *= 2
    return p


# line-fast compile-time shapes (fft_device.hpp CtShapeSel<T, N, S, true>): N -> (E, radices, budget, maxThr)
LF_SHAPES = {
    8: {16: (16, (16,), 65536, 256), 32: (8, (8, 4), 65536, 256), 64: (8, (8, 8), 65536, 256),
        128: (16, (16, 8), 65536, 256), 256: (16, (16, 16), 65536, 256),
        512: (16, (16, 16, 2), 81920, 512), 1024: (32, (16, 16, 4), 153600, 512)},
    16: {16: (16, (16,), 65536, 256), 32: (8, (8, 4), 65536, 256), 64: (8, (8, 8), 65536, 256),
         128: (8, (8, 8, 2), 65536, 256), 256: (8, (8, 8, 4), 65536, 256),
         512: (8, (8, 8, 8), 81920, 512), 1024: (16, (16, 16, 4), 153600, 512)},
}


def lf_cases():
    for eb, shapes in LF_SHAPES.items():
        for n, (e, rad, budget, thr) in shapes.items():
            tp = n // e
            b0 = lines_per_block(tp, padded_stride(n, eb) * eb, budget, thr)
            yield eb, n, e, rad, lf_lines(b0)


def residue_table():
    for eb, n, e, rad, b in lf_cases():
        kmod = 32 if eb == 8 else 16
        lo = min_stride(n, eb)
        res = {}
        for ls in range(lo, lo + kmod):
            res[ls % kmod] = cycles_for_stride(n, e, rad, b, eb, ls)[0]
        cur = current_stride(n, b, eb)
        best = min(res.values())
        print(f"eb={eb} N={n} E={e} B={b} cur%{kmod}={cur % kmod}:{res[cur % kmod]} best={best} "
              f"residues={[r for r, c in sorted(res.items()) if c == best]}", flush=True)


def accesses(N, E, radices, B, shift, lf):
    """LDS accesses of one FftCT workgroup: first-pass reads, the exchanges between
    passes, the result write; lf: line-fast lane mapping (else row-mapped)."""
    TP = N // E
    NT = B * TP
    pad = lambda i: i + (i >> shift)
    out = []
    rs = [r for r in radices if r > 1]

    def lanes():
        for tid in range(NT):
            yield (tid, tid % B, tid // B) if lf else (tid, tid // TP, tid % TP)

    def reads(R):
        for k in range(E // R):
            for r in range(R):
                out.append((False, {tid: (b, pad(t + k * TP + r * (N // R))) for tid, b, t in lanes()}))

    reads(rs[0])
    ns = 1
    for i in range(len(rs) - 1):
        R, RN = rs[i], rs[i + 1]
        for k in range(E // R):
            for r in range(R):
                acc = {}
                for tid, b, t in lanes():
                    j = t + k * TP
                    kk = j % ns
                    acc[tid] = (b, pad((j - kk) * R + kk + r * ns))
                out.append((True, acc))
        reads(RN)
        ns *= R
    RL = rs[-1]
    for k in range(E // RL):
        for r in range(RL):
            out.append((True, {tid: (b, pad(t + k * TP + r * (N // RL))) for tid, b, t in lanes()}))
    return out, NT


def workgroup_cycles(N, E, radices, B, eb, LS, shift, lf):
    accs, NT = accesses(N, E, radices, B, shift, lf)
    tot = ideal = 0
    for w in range(NT // 64):
        for write, acc in accs:
            addrs = {tid - 64 * w: eb * (b * LS + p) for tid, (b, p) in acc.items()
                     if 64 * w <= tid < 64 * (w + 1)}
            tot += access_cycles(addrs, eb, write)
            ideal += 4 if eb == 8 else (8 if write else 4)
    return tot, ideal


def new_lf_stride(n, b, eb, shift):
    """fft_device.hpp lf_padded_stride (round 4)."""
    ls = n + ((n - 1) >> shift) + 1
    if eb == 16 and b == 8:
        while ls % 16 not in (7, 9):
            ls += 1
        return ls
    mm = 1 if b >= 16 else (16 if eb == 8 else 8) // b
    while ls % (2 * mm) != mm:
        ls += 1
    return ls


def compare():
    """Old (pad per 256 B, lf stride == kMod/B) vs new (fp32 pad per 128 B, new lf
    strides) LDS cycles of the compile-time engines, line-fast and row-mapped."""
    for eb, shapes in LF_SHAPES.items():
        for n, (e, rad, budget, thr) in shapes.items():
            tp = n // e
            b = lf_lines(lines_per_block(tp, padded_stride(n, eb) * eb, budget, thr))
            old = workgroup_cycles(n, e, rad, b, eb, current_stride(n, b, eb), 5 if eb == 8 else 4, True)
            new = workgroup_cycles(n, e, rad, b, eb, new_lf_stride(n, b, eb, 4), 4, True)
            print(f"LF  eb={eb:2d} N={n:4d} B={b:2d}: old {old[0]:6d} new {new[0]:6d} ideal {old[1]:6d}",
                  flush=True)
