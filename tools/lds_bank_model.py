#!/usr/bin/env python3
"""LDS bank-conflict model of the MI355X lane groups (MI355X_MICROARCH.md, LDS table), used to
pick the LDS layouts of the fused conv kernels (csrc/kernels/cnn_fused.hip).

    ds_read_b128        4 groups of 16 lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... ;
                        16 B per lane, bank = (byte address / 4) mod 64
    ds_read_b64_tr_b16  2 groups of 32 lanes; 8 B per lane, bank = (byte address / 4) mod 64

A group costs one LDS cycle per distinct address on its busiest bank; the numbers printed
are LDS cycles per conflict-free cycle (1.0 = conflict-free).

    python tools/lds_bank_model.py            # conv3 backward: old vs shipped layouts
    python tools/lds_bank_model.py --search   # the conv3 layout / swizzle search behind them
    python tools/lds_bank_model.py --conv2    # the conv2 backward images
    python tools/lds_bank_model.py --fwd      # the fused forward's frame / a1 / a2 images

A model, not a clock: the swizzled layouts it prefers need per-read XOR address arithmetic,
which in these two-waves-per-SIMD kernels cost more than the conflicts they removed
(profiles/r4_cnn_swizzle_ab.txt); the shipped layouts are the padding-only ones.
"""
import sys

G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
        list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
        list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]
G64 = [list(range(32)), list(range(32, 64))]


def _cycles(addr, groups, dwords):
    tot = 0
    for grp in groups:
        banks = {}
        for lane in grp:
            a = addr[lane] // 4
            for d in range(dwords):
                banks.setdefault((a + d) % 64, set()).add(a + d)
        tot += max(len(s) for s in banks.values())
    return tot


def b128(addr):
    return _cycles(addr, G128, 4) / 4


def tr16(addr):
    return _cycles(addr, G64, 2) / 2


def lanes():
    for lane in range(64):
        yield lane & 15, lane >> 4, (lane >> 2) & 3, lane & 3  # i16, g, q4, p4


def swz(row_fn, ld, f):
    """element address of (image row, channel) with the 16-byte chunk XOR swizzle f(row)"""
    def el(y, x, col):
        r = row_fn(y, x)
        return r * ld + ((((col >> 3) ^ f(y, x)) & 7) << 3) + (col & 7)
    return el


def conv3_bwd_da3(el):
    """(dgrad b128 factor, wgrad transposed factor, LDS cycles per wave-image) of the da3 image"""
    rd, rw = [], []
    for half in (0, 1):
        for u in range(3):
            for ks in range(18):
                t = ks >> 1
                kh, kw = t // 3, t % 3
                addr = []
                for i16, g, q4, p4 in lanes():
                    p = 16 * (3 * half + u) + i16
                    pc = p if p < 81 else 0
                    addr.append(2 * el(pc // 9 + 2 - kh, pc % 9 + 2 - kw, (ks & 1) * 32 + 8 * g))
                rd.append(b128(addr))
    for s in (0, 1):
        for c in range(4):
            for hi in (0, 1):
                addr = [2 * el(4 * s + g + 2, 2 + q4 + 4 * hi, 16 * c + 4 * p4) for i16, g, q4, p4 in lanes()]
                rw.append(tr16(addr))
    d, w = sum(rd) / len(rd), sum(rw) / len(rw)
    return round(d, 2), round(w, 2), 54 * 4 * d + 16 * 2 * w


def conv3_bwd_a2(el):
    """(wgrad transposed factor, LDS cycles per wave-image) of the a2 image"""
    rw = []
    for s in (0, 1):
        for half in (0, 1):
            for t in range(5):
                for ct in range(4):
                    for hi in (0, 1):
                        tap = min(half * 5 + t, 8)
                        kh, kw = tap // 3, tap % 3
                        addr = [2 * el(4 * s + g + kh, kw + q4 + 4 * hi, 16 * ct + 4 * p4) for i16, g, q4, p4 in lanes()]
                        rw.append(tr16(addr))
    w = sum(rw) / len(rw)
    return round(w, 2), 20 * 2 * w


def main():
    none = lambda y, x: 0  # noqa: E731
    old_y = swz(lambda y, x: y * 11 + x, 72, none)
    old_x = swz(lambda y, x: y * 9 + x, 72, none)
    new_y = swz(lambda y, x: y * 11 + x, 80, none)
    swz_y = swz(lambda y, x: y * 11 + x, 64, lambda y, x: y + x)
    new_x = swz(lambda y, x: y * 12 + x, 80, none)
    print("conv3_bwd da3 image (dgrad b128, wgrad tr, cycles):  old 11-wide/72 ->", conv3_bwd_da3(old_y),
          " shipped 11-wide/80 ->", conv3_bwd_da3(new_y), " swizzled 11-wide/64 + chunk ^ (y + x) (measured no",
          "faster: its address arithmetic) ->", conv3_bwd_da3(swz_y))
    print("conv3_bwd a2 image (wgrad tr, cycles):                old 9-wide/72 ->", conv3_bwd_a2(old_x),
          " shipped 12-wide/80 ->", conv3_bwd_a2(new_x))
    if "--conv2" in sys.argv:
        search_conv2()
    if "--fwd" in sys.argv:
        print("conv_stack_fwd conv1 frame reads (ld, row width -> factor):",
              {(ld, W): conv_stack_fwd_conv1(ld, W) for ld in (72, 80, 88) for W in (21, 24, 28, 32)})
        print("conv_stack_fwd conv2 a1 reads (ld -> factor): stride-2 rows of 20",
              {ld: conv_stack_fwd_conv2(ld, False) for ld in (40, 48, 56)}, " 9 x 10 grid on phase images",
              {ld: conv_stack_fwd_conv2(ld, True) for ld in (40, 48, 56)})
        print("conv_stack_fwd conv3 a2 reads (ld -> factor): 49 pixels", {ld: conv_stack_fwd_conv3(ld, False) for ld in (72, 80)},
              " 7 x 9 grid", {ld: conv_stack_fwd_conv3(ld, True) for ld in (72, 80)})
    if "--search" in sys.argv:
        res = []
        for ld in (64, 72, 80, 88):
            for W in (11, 12, 13, 16):
                for a in range(8):
                    for b in range(8):
                        f = (lambda y, x, a=a, b=b: a * x + b * y)
                        d, w, c = conv3_bwd_da3(swz(lambda y, x, W=W: y * W + x, ld, f))
                        res.append((round(c, 1), ld, W, f"chunk ^ ({a} x + {b} y)", d, w))
        res.sort()
        print("da3 image, best layouts:")
        for r in res[:6]:
            print("  ", r)
        res = []
        for ld in (64, 72, 80):
            for W in (9, 10, 11, 12, 13, 16):
                for name, f in (("none", none), ("y&7", lambda y, x: y), ("x&7", lambda y, x: x)):
                    w, c = conv3_bwd_a2(swz(lambda y, x, W=W: y * W + x, ld, f))
                    res.append((round(c, 1), ld, W, name, w))
        res.sort()
        print("a2 image, best layouts:")
        for r in res[:6]:
            print("  ", r)


def conv2_bwd_da2(el, grid12=False):
    """(dgrad b128, wgrad transposed, LDS cycles per wave-image) of the da2 image; el(y, x, col)
    addresses bordered position (y, x) = (oh + 1, ow + 1).  grid12: each phase class's 10 x 10
    dgrad pixels computed as a 10 x 12 grid, 8 tiles (the shipped form) instead of 7"""
    rd, rw = [], []
    W = 12 if grid12 else 10
    for cls in range(4):
        for T0, NT in ((0, 4), (4, 4 if grid12 else 3)):
            for u in range(NT):
                for ks in range(8):
                    t = ks >> 1
                    ti, tj = t >> 1, t & 1
                    addr = []
                    for i16, g, q4, p4 in lanes():
                        p = 16 * (T0 + u) + i16
                        pc = p if (p < 100 or grid12) else 0
                        addr.append(2 * el(pc // W + 1 - ti, pc % W + 1 - tj, (ks & 1) * 32 + 8 * g))
                    rd.append(b128(addr))

    def run(s, g, h):
        R = 2 * (4 * s + g) + h
        return (R // 3, 4 * (R % 3)) if R < 27 else (9, 0)
    for s in range(4):
        for c in range(4):
            for h in (0, 1):
                addr = []
                for i16, g, q4, p4 in lanes():
                    oh, ow0 = run(s, g, h)
                    addr.append(2 * el(oh + 1, ow0 + 1 + q4, 16 * c + 4 * p4))
                rw.append(tr16(addr))
    d, w = sum(rd) / len(rd), sum(rw) / len(rw)
    # per wave-image: dgrad 7 (8) tiles x 8 k-steps b128 (4 cycles), wgrad 4 x 4 x 2 transposed (2 cycles)
    return round(d, 2), round(w, 2), (64 if grid12 else 56) * 4 * d + 32 * 2 * w


def conv2_bwd_a1(el):
    """(wgrad transposed, LDS cycles per wave-image) of the a1 phase images; el(phase, y, x, col)"""
    rw = []

    def run(s, g, h):
        R = 2 * (4 * s + g) + h
        return (R // 3, 4 * (R % 3)) if R < 27 else (9, 0)
    for s in range(4):
        for w in range(8):
            cb, tau0 = w & 1, 4 * (w >> 1)
            for t in range(4):
                tau = tau0 + t
                kh, kw = tau >> 2, tau & 3
                for h in (0, 1):
                    addr = []
                    for i16, g, q4, p4 in lanes():
                        oh, ow0 = run(s, g, h)
                        addr.append(2 * el((kh & 1) * 2 + (kw & 1), oh + (kh >> 1), ow0 + (kw >> 1) + q4, 16 * cb + 4 * p4))
                    rw.append(tr16(addr))
    w = sum(rw) / len(rw)
    return round(w, 2), 32 * 2 * w


def search_conv2():
    none = lambda y, x: 0  # noqa: E731
    print("conv2_bwd da2 image (dgrad b128, wgrad tr, cycles): 12-wide/72 ->",
          conv2_bwd_da2(swz(lambda y, x: y * 12 + x, 72, none)), " 12-wide/80 ->",
          conv2_bwd_da2(swz(lambda y, x: y * 12 + x, 80, none)), " 12-wide/80, 10 x 12 dgrad grid (shipped) ->",
          conv2_bwd_da2(swz(lambda y, x: y * 12 + x, 80, none), grid12=True))
    res = []
    for ld in (64, 72, 80):
        for W in (12, 13, 14, 16):
            for a in range(8):
                for b in range(8):
                    f = (lambda y, x, a=a, b=b: a * x + b * y)
                    d, w, c = conv2_bwd_da2(swz(lambda y, x, W=W: y * W + x, ld, f))
                    res.append((round(c, 1), ld, W, f"chunk ^ ({a} x + {b} y)", d, w))
    res.sort()
    for r in res[:6]:
        print("  ", r)

    def a1el(W, ld, rows, f):
        def el(ph, y, x, col):
            r = ph * rows + y * W + x
            return r * ld + ((((col >> 3) ^ f(y, x)) & 3) << 3) + (col & 7)
        return el
    print("conv2_bwd a1 phase images (wgrad tr, cycles): current 10-wide/40 ->", conv2_bwd_a1(a1el(10, 40, 116, none)))
    res = []
    for ld in (32, 40, 48, 56):
        for W in (10, 11, 12, 16):
            rows = max(116, ((11 * W + 15) // 16) * 16)
            for a in range(4):
                for b in range(4):
                    f = (lambda y, x, a=a, b=b: a * x + b * y)
                    w, c = conv2_bwd_a1(a1el(W, ld, rows, f))
                    res.append((round(c, 1), ld, W, rows, f"chunk ^ ({a} x + {b} y)", w))
    res.sort()
    for r in res[:6]:
        print("  ", r)


def conv_stack_fwd_conv1(ld, W):
    """b128 factor of conv1's frame fragment reads, frame positions (a, b) at LDS row W a + b"""
    r = []
    for t in range(25):
        for ks in range(8):
            tap = ks >> 1
            addr = []
            for i16, g, q4, p4 in lanes():
                p = 16 * t + i16
                row = (p // 20 + (tap >> 1)) * W + p % 20 + (tap & 1)
                addr.append(2 * (row * ld + 32 * (ks & 1) + 8 * g))
            r.append(b128(addr))
    return round(sum(r) / len(r), 2)


def conv_stack_fwd_conv2(ld, grid10):
    """b128 factor of the fused forward's conv2 reads of a1: grid10=False -- 81 output pixels
    read from the 20 x 20 image in rows of 20 (stride-2 positions); True -- a 9 x 10 grid
    (column 9 discarded) read from four stride-2 phase images of 100 rows (the shipped form)"""
    r = []
    for t in range(6):
        for ks in range(16):
            kh, kw = ks >> 2, ks & 3
            addr = []
            for i16, g, q4, p4 in lanes():
                p = 16 * t + i16
                if grid10:
                    oh, ow = p // 10, p % 10
                    row = ((kh & 1) * 2 + (kw & 1)) * 100 + (oh + (kh >> 1)) * 10 + ow + (kw >> 1)
                else:
                    pc = p if p < 81 else 0
                    row = 2 * (pc // 9) * 20 + 2 * (pc % 9) + kh * 20 + kw
                addr.append(2 * (row * ld + 8 * g))
            r.append(b128(addr))
    return round(sum(r) / len(r), 2)


def conv_stack_fwd_conv3(ld, grid9):
    """b128 factor of the fused forward's conv3 reads of a2 (9 x 9 image, rows of 9): grid9=False
    -- 49 output pixels; True -- a 7 x 9 grid (columns 7, 8 discarded, the shipped form)"""
    r = []
    for t in range(4):
        for ks in range(18):
            tap = ks >> 1
            kh, kw = tap // 3, tap % 3
            addr = []
            for i16, g, q4, p4 in lanes():
                p = 16 * t + i16
                if grid9:
                    row = p + kh * 9 + kw
                else:
                    pc = p if p < 49 else 0
                    row = (pc // 7) * 9 + pc % 7 + kh * 9 + kw
                addr.append(2 * (row * ld + 32 * (ks & 1) + 8 * g))
            r.append(b128(addr))
    return round(sum(r) / len(r), 2)


if __name__ == "__main__":
    main()
