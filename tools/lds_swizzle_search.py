"""Search a linear XOR swizzle f(column) for the fast kernels' LDS tile so that
every access pattern of kernels_fast.hip is bank-conflict free (bank rules:
MI355X_MICROARCH.md §LDS).  Prints the matrix rows (one 5-bit mask per column bit)."""
import random, sys

TILE = 256
B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[x + 32 for x in g] for g in B128_GROUPS]


def make_B(K, A):
    Q = K // 4
    P = max(1, 32 // Q)
    W = max(32, Q)
    def f(cs):
        v = 0
        for bit, row in enumerate(A):
            if (cs >> bit) & 1:
                v ^= row
        return v
    def B(c, m):
        cs, ci = divmod(c, P)
        return cs * W + ((ci * Q + m) ^ f(cs))
    return B


def ok(K, A):
    B = make_B(K, A)
    Q, R = K // 4, K // 64
    # bijectivity
    seen = set(B(c, m) for c in range(TILE) for m in range(Q))
    if len(seen) != TILE * Q:
        return False
    for g in range(Q // 4):
        for u in range(4):
            for i in range(4):
                addr = [B(4 * l + i, 4 * g + u) for l in range(64)]
                for h in range(2):  # ds_read_b64
                    if len({a % 32 for a in addr[32 * h:32 * h + 32]}) != 32:
                        return False
                for q in range(4):  # ds_write_b64
                    if len({a % 16 for a in addr[16 * q:16 * q + 16]}) != 16:
                        return False
    nthreads = 4 * K
    for j in range(Q // R):
        for w in range(nthreads // 64):
            addr = [B((64 * w + l) // R, R * j + (64 * w + l) % R) for l in range(64)]
            for h in range(2):
                if len({a % 32 for a in addr[32 * h:32 * h + 32]}) != 32:
                    return False
            for q in range(4):  # K=64: 2-way on these writes is unavoidable (2 columns per 128 B)
                if K > 64 and len({a % 16 for a in addr[16 * q:16 * q + 16]}) != 16:
                    return False
    # 8-byte row-major sweeps (tile load / copy-out): thread t -> block t
    for w in range(TILE * Q // 64):
        addr = [B(*divmod(64 * w + l, Q)) for l in range(64)]
        for h in range(2):
            if len({a % 32 for a in addr[32 * h:32 * h + 32]}) != 32:
                return False
        for q in range(4):
            if len({a % 16 for a in addr[16 * q:16 * q + 16]}) != 16:
                return False
    return True


def search(K, tries=20000, seed=1):
    rng = random.Random(seed)
    Q = K // 4
    P = max(1, 32 // Q)
    nbits = (TILE // P - 1).bit_length()
    width = min(32, max(32, Q)) if Q < 32 else 32
    for _ in range(tries):
        A = [rng.randrange(0, 32) for _ in range(nbits)]
        if ok(K, A):
            return A
    return None


if __name__ == "__main__":
    for K in (64, 128, 256):
        A = search(K)
        print(K, A)
