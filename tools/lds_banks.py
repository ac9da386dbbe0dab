"""LDS bank-conflict simulator for gfx950 (rules: MI355X_MICROARCH.md §LDS).

Used to pick the XOR swizzles of the GEMM / attention LDS images before
writing the HIP code.  cost = LDS cycles per wave-instruction (ideal: 4 for
ds_read_b128, 2 for ds_read_b64 / ds_read_b64_tr_b16).
"""
from collections import defaultdict

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]
HALF_GROUPS = [list(range(0, 32)), list(range(32, 64))]


def cost(addrs, nbytes, groups):
    total = 0
    for g in groups:
        banks = defaultdict(set)
        for l in g:
            a = addrs[l]
            for d in range(nbytes // 4):
                dw = a // 4 + d
                banks[dw % 64].add(dw)
        total += max(len(s) for s in banks.values())
    return total


def gemm_a_read(swz, row_bytes=128, ks=0):
    # 16x16x32 bf16 operand: lane l reads row l&15, 16-B chunk 4*ks + (l>>4)
    addrs = []
    for l in range(64):
        r, c = l & 15, 4 * ks + (l >> 4)
        addrs.append(r * row_bytes + 16 * swz(r, c))
    return cost(addrs, 16, B128_GROUPS)


def attn_v_tr_read(swz, ks=0, dt=0, second=0):
    # ds_read_b64_tr_b16: group g = l>>4, lane i=l&15 -> 4q+p supplies row q, cols 4p..4p+3
    addrs = []
    for l in range(64):
        g, i = l >> 4, l & 15
        q, p = i >> 2, i & 3
        key = 32 * ks + 16 * second + 4 * g + q
        col = 16 * dt + 4 * p                  # bf16 element index
        chunk, half = col // 8, (col % 8) // 4
        addrs.append(key * 256 + 16 * swz(key, chunk) + 8 * half)
    return cost(addrs, 8, HALF_GROUPS)


if __name__ == "__main__":
    ident = lambda r, c: c
    cands = {
        "none": ident,
        "c^(r&7)": lambda r, c: c ^ (r & 7),
        "c^((r>>1)&7)": lambda r, c: c ^ ((r >> 1) & 7),
    }
    for n, f in cands.items():
        print("GEMM 128B rows", n, [gemm_a_read(f, 128, ks) for ks in (0, 1)])
    cands256 = {
        "none": ident,
        "c^(r&15)": lambda r, c: c ^ (r & 15),
        "c^((r&3)<<2|(r>>2)&3)": lambda r, c: c ^ (((r & 3) << 2) | ((r >> 2) & 3)),
    }
    for n, f in cands256.items():
        print("ATTN K 256B rows", n, [gemm_a_read(f, 256, ks) for ks in range(4)],
              "V tr", [attn_v_tr_read(f, ks, dt, s) for ks in (0, 1) for dt in (0, 3) for s in (0, 1)])


def search_64B_rows():
    """256 x 32 bf16 k-half pieces: 64-B rows, 4 x 16-B chunks per row."""
    import itertools
    best = []
    for a, b, c in itertools.product(range(4), repeat=3):
        # g(r) = linear combination of bit-pairs of the row index
        def swz(r, ch, a=a, b=b, c=c):
            g = (((r >> 2) & 3) * a + ((r >> 4) & 3) * b + (r & 3) * c) & 3
            return ch ^ g
        costs = []
        for t in range(4):                       # 4 row-tiles of 16 rows
            addrs = []
            for l in range(64):
                r, ch = 16 * t + (l & 15), l >> 4
                addrs.append(r * 64 + 16 * swz(r, ch))
            costs.append(cost(addrs, 16, B128_GROUPS))
        best.append((max(costs), (a, b, c)))
    best.sort()
    return best[:5]
