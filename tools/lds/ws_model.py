"""LDS model of conv_fwd_bs_ws_kernel (csrc/conv.hip): bank cycles of every LDS access of
one four-chunk frame (MI355X_MICROARCH.md §LDS rules, banks.py) and a symbolic check that
each lane's A and B fragments pair the same (chunk, tap, channel) in every k-element.

usage: python tools/lds/ws_model.py [TH TW]  (default: the conv3_3 tiles 30x17, 15x34, 13x39)
Mirrors the kernel's address arithmetic; the round-4 layout (one ds_read_b128 per B unit,
pitch TW + 2) is modelled for comparison with --old."""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import banks  # noqa: E402

NPL, BM, AROW, ALLOC = 3, 64, 160, 1056


def pitch(tw):
    return tw + 2 if tw % 16 == 0 else tw + 16


def cfg(old):
    a_plane = BM * AROW
    b_plane = (640 if old else ALLOC) * 16
    buf0 = NPL * (a_plane + b_plane)
    buf = buf0 + 16 if (buf0 // 16) % 2 == 0 else buf0
    return a_plane, b_plane, buf


def frame(TH, TW, old=False):
    """LDS cycles / conflict-free cycles of the MFMA waves' fragment reads over one frame,
    and the producers' stores; plus the fragment pairing check."""
    A_PLANE, B_PLANE, BUF = cfg(old)
    PW = TW + 2
    PS = PW if old else pitch(TW)

    def tap_c(t):
        return ((t // 3) * PS + t % 3) * 16

    def ua(u):
        return (BUF if u >= 9 else 0) + 16 * (u % 9)

    def ub(u):
        return (BUF if u >= 9 else 0) + tap_c(u % 9)

    # symbolic LDS contents: byte address -> (kind, chunk-in-buffer-pair, tap/pos, channel)
    a_cont, b_cont = {}, {}
    for S in range(2):  # weights: row r, tap slot q, channels 8 -> 16 B (2 B each)
        for q in range(10):
            swap = (q + S) % 2 == 1 and not old
            for e in range(8):
                e_st = (e + 4) % 8 if swap else e
                for r in range(16):
                    a_cont[S * BUF + r * AROW + 16 * q + 2 * e_st] = (S, q, e)
    for S in range(2):  # input patch position (pr, pc), channel e
        for pr in range(TH + 2):
            for pc in range(PW):
                for e in range(8):
                    b_cont[S * BUF + NPL * A_PLANE + (pr * PS + pc) * 16 + 2 * e] = (S, pr, pc, e)
    cyc = ideal = 0
    for wn in range(8):
        for cb in range(4):
            for s in range(9):
                a_addr, b_lo, b_hi = [], [], []
                for lane in range(64):
                    l16, g = lane & 15, lane >> 4
                    u = (4 * s + g) % 18
                    q = (wn * 64 + cb * 16 + l16) % (TH * TW)
                    hb = 0 if old else 8 * (g & 1)
                    bp = NPL * A_PLANE + ((q // TW) * PS + q % TW) * 16 + hb
                    a_addr.append(l16 * AROW + ua(u))
                    b0 = bp + ub(u)
                    b_lo.append(b0)
                    b_hi.append(b0 ^ 8)
                    if cb == 0 and wn == 0 or not old and s < 2:
                        # pairing check: A k-element j and B k-element j
                        for j in range(8):
                            aj = a_cont[a_addr[-1] + 2 * j]
                            bj = b_cont[(b0 if j < 4 else b0 ^ 8) + 2 * (j % 4)] if not old else \
                                b_cont[b0 + 2 * j]
                            tap = u % 9
                            qr, qc = q // TW, q % TW
                            assert aj == (u // 9, tap, bj[3]), (aj, bj)
                            assert bj[:3] == (u // 9, qr + tap // 3, qc + tap % 3), (bj, u, q)
                if cb == 0:  # A: 4 row blocks x NPL planes per step (same banks per block)
                    cyc += banks.read_b128(a_addr) * 4 * NPL
                    ideal += 4 * 4 * NPL
                if old:
                    cyc += banks.read_b128(b_lo) * NPL
                    ideal += 4 * NPL
                else:
                    cyc += (banks.read_b64(b_lo) + banks.read_b64(b_hi)) * NPL
                    ideal += 4 * NPL
    # producers' B stores: positions ptid + 256 i, ds_write_b128
    st = st_ideal = 0
    PP = (TH + 2) * PW
    for i in range(3):
        addrs = []
        for ptid in range(256):
            pos = min(ptid + 256 * i, PP - 1)
            addrs.append(NPL * A_PLANE + ((pos // PW) * PS + pos % PW) * 16)
        for w in range(4):
            st += banks.write_b128(addrs[64 * w:64 * w + 64])
            st_ideal += 8
    return cyc / ideal, st / st_ideal


if __name__ == "__main__":
    old = "--old" in sys.argv
    args = [int(a) for a in sys.argv[1:] if a.isdigit()]
    tiles = [tuple(args[:2])] if args else [(30, 17), (15, 34), (13, 39), (16, 32)]
    for th, tw in tiles:
        r, w = frame(th, tw, old)
        print(f"{'old' if old else 'new'} {th}x{tw}: fragment reads {r:.3f}x conflict-free, "
              f"patch stores {w:.3f}x")
