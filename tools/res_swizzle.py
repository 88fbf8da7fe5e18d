"""Bank-conflict check / search of the resident kernels' LDS swizzle
(kernels_res.hip rsw): 8-byte position-quad items of column c, block m at
2K c + 8 (m ^ rsw(c)), rsw linear in the bits of c.  Bank rules
(MI355X_MICROARCH.md §LDS): ds_read_b64 in 32-lane groups over 64 banks,
ds_write_b64 in 16-lane groups over 32 banks, i.e. items distinct mod 32 /
mod 16.  Sweeps: CQ (read/write), HA (read/write), HD (read/write), the
payload tile's natural-block writes.  Usage: python tools/res_swizzle.py
[K ...] -> checks the product swizzle of each K, searches one if it fails."""
import random
import sys


def rsw_of(rows):
    def f(c):
        v = 0
        for b, r in enumerate(rows):
            if (c >> b) & 1:
                v ^= r
        return v
    return f


def sweeps(K):
    W = K // 64          # waves
    LPC = K // 64        # HD lanes per column
    CPW = 64 // LPC      # HD columns per wave
    out = []             # (kind, [(c, m) per lane])
    for w in range(W):
        for e in range(4):
            for q in range(4):
                out.append(("rw", [(4 * (l & 15) + e, 16 * w + 4 * (l >> 4) + q) for l in range(64)]))
        for j in range(16):
            out.append(("rw", [(l, (w & 3) + 4 * j + 64 * (w >> 2)) for l in range(64)]))
            out.append(("rw", [(CPW * w + l // LPC, l % LPC + LPC * j) for l in range(64)]))
        for i in range(16):
            lanes = []
            for l in range(64):
                t = 64 * w + l
                lanes.append((t // (K // 4) + 4 * i, t % (K // 4)))
            out.append(("w", lanes))
    return out


def conflicts(K, f):
    bad = 0
    for kind, lanes in sweeps(K):
        items = [m ^ f(c) for c, m in lanes]  # column offsets 2K c are 0 mod every bank count
        for h in range(2):
            if kind == "rw" and len({x % 32 for x in items[32 * h:32 * h + 32]}) != 32:
                bad += 1
        for g in range(4):
            if len({x % 16 for x in items[16 * g:16 * g + 16]}) != 16:
                bad += 1
    return bad


PRODUCT = {1024: [24, 4, 1, 2, 20, 8], 512: [28, 14, 1, 25, 20, 27], 256: [24, 4, 14, 5, 17, 23]}  # kernels_res rsw<K>


# The encode's quad items (res_common.hpp Qi): column quad cq at position p,
# item index 16 pi(p) + cq with pi(p) = p ^ ((p >> 4) & 1) (pi_bit = 4), or
# the identity (pi_bit = None).  Sweeps: CQ (lane 16 u + cq, p = 64 w + 16 u
# + i), HA' (p = (w >> 2) << 8 | j << 4 | (w & 3) << 2 | a), HD' (p = j <<
# (logK - 4) | w << 2 | a), a = lane >> 4.
def qi_sweeps(K):
    W, logk = K // 64, K.bit_length() - 1
    out = []
    for w in range(W):
        for i in range(16):
            out.append([(l & 15, 64 * w + 16 * (l >> 4) + i) for l in range(64)])
            out.append([(l & 15, ((w >> 2) << 8) | (i << 4) | ((w & 3) << 2) | (l >> 4)) for l in range(64)])
            out.append([(l & 15, (i << (logk - 4)) | (w << 2) | (l >> 4)) for l in range(64)])
    return out


def qi_conflicts(K, pi_bit=4):
    def pi(p):
        return p if pi_bit is None else p ^ ((p >> pi_bit) & 1)
    bad = 0
    for lanes in qi_sweeps(K):
        items = [16 * pi(p) + cq for cq, p in lanes]
        assert len(set(items)) == 64 and max(items) < 16 * K
        for h in range(2):
            if len({x % 32 for x in items[32 * h:32 * h + 32]}) != 32:
                bad += 1
        for g in range(4):
            if len({x % 16 for x in items[16 * g:16 * g + 16]}) != 16:
                bad += 1
    return bad


def search(K, tries=200000, seed=1):
    rng = random.Random(seed)
    top = K // 4
    for _ in range(tries):
        rows = [rng.randrange(0, min(top, 32)) for _ in range(6)]
        if conflicts(K, rsw_of(rows)) == 0:
            return rows
    return None


if __name__ == "__main__":
    for K in [int(a) for a in sys.argv[1:]] or [1024, 512, 256]:
        rows = PRODUCT.get(K)
        if rows is not None:
            print(K, rows, "conflicting wave-instruction groups:", conflicts(K, rsw_of(rows)))
        else:
            print(K, "search:", search(K))
        print(K, "encode quad items, conflicting wave-instruction groups:", qi_conflicts(K))
