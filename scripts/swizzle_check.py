"""Brute-force bank-conflict and invariance check of the LDS images of wgrad3x3_pipe_kernel (dmc_conv.hip):

  * the x halo (swz_h<OW>): for every tap, k-step, fragment half and 32-lane group, the 8-byte reads of
    ds_read_b64_tr_b16 hit 64 distinct banks ((byte / 4) mod 64, two dwords per lane);
  * every read of an address set equals base + immediate: the swizzle of the rows a set serves (tap rows of one
    row class, all k-steps) is the swizzle of the set's base row;
  * the dy ring image (swz_x, 128-byte rows): the same conflict check, and k-step 1 = k-step 0 + 32 rows.

    python scripts/swizzle_check.py
"""
import sys


def geo(OW):
    TILE = 128 if OW >= 8 else 64
    R = 128 // OW if OW >= 16 else OW
    NIMG = 1 if OW >= 16 else TILE // (OW * OW)
    HW = OW + 2
    SEGP = (R + 2) * HW
    set_of = (lambda ty: 0) if OW >= 16 else (lambda ty: ty & 1) if OW == 8 else (lambda ty: ty)

    def hrow(p):
        return (p // (R * OW)) * SEGP + ((p % (R * OW)) // OW + 1) * HW + (p % OW) + 1

    def swz(h):
        hc, hr = h % HW, h // HW
        b1 = (hc >> 3) & 1 if OW >= 16 else (hr & 1) if OW == 8 else (hr >> 1) & 1
        return ((hc >> 1) & 1) | (b1 << 1)
    return TILE, HW, hrow, swz, set_of


def lane_fields(lane):
    return lane >> 4, (lane >> 2) & 3, lane & 3      # fh, q, pcol


def check_x(OW):
    TILE, HW, hrow, swz, set_of = geo(OW)
    bad = 0
    for wq in range(4):                                  # segment of the wave
        for ty in range(3):
            for tx in range(3):
                py = set_of(ty)
                for j in range(TILE // 32):
                    for hf in range(2):
                        addrs = []
                        for lane in range(64):
                            fh, q, pcol = lane_fields(lane)
                            h = hrow(32 * j + 8 * fh + 4 * hf) + q + (ty - 1) * HW + (tx - 1)
                            a = h * 128 + ((wq ^ swz(h)) << 5) + pcol * 8
                            # the kernel's form: the set's base row (k-step 0, row class py) + immediate
                            hb = hrow(8 * fh + 4 * hf) + q + (py - 1) * HW + (tx - 1)
                            ab = hb * 128 + ((wq ^ swz(hb)) << 5) + pcol * 8
                            imm = (hrow(32 * j) - hrow(0)) * 128 + (ty - py) * HW * 128
                            if ab + imm != a:
                                bad += 1
                            addrs.append(a)
                        for g in (range(32), range(32, 64)):
                            banks = {}
                            for lane in g:
                                for d in range(2):
                                    b = (addrs[lane] // 4 + d) % 64
                                    w = addrs[lane] // 4 + d
                                    if banks.get(b, w) != w:
                                        bad += 1
                                    banks[b] = w
    return bad


def check_dy():
    def swz_x(row):
        return ((row >> 1) & 1) | (((row >> 3) & 1) << 1)
    bad = 0
    for ks in range(2):
        for i in range(4):
            for hf in range(2):
                addrs = []
                for lane in range(64):
                    fh, q, pcol = lane_fields(lane)
                    row = ks * 32 + 8 * fh + 4 * hf + q
                    a = row * 128 + ((i ^ swz_x(row)) << 5) + pcol * 8
                    r0 = 8 * fh + 4 * hf + q
                    if r0 * 128 + ((i ^ swz_x(r0)) << 5) + pcol * 8 + ks * 4096 != a:
                        bad += 1
                    addrs.append(a)
                for g in (range(32), range(32, 64)):
                    banks = {}
                    for lane in g:
                        for d in range(2):
                            b = (addrs[lane] // 4 + d) % 64
                            w = addrs[lane] // 4 + d
                            if banks.get(b, w) != w:
                                bad += 1
                            banks[b] = w
    return bad


if __name__ == "__main__":
    total = 0
    for OW in (32, 16, 8, 4):
        n = check_x(OW)
        print(f"x halo OW={OW}: {n} violations")
        total += n
    n = check_dy()
    print(f"dy ring: {n} violations")
    total += n
    sys.exit(1 if total else 0)
