"""numpy model of conv1's input gradient on 2:4-sparse 16x16x64 MFMA fragments (the layout
ba3c_dgrad2s.h implements), checked against the dense input gradient of the un-pooled dY.
Lane layouts (scripts/probes/smfmac_probe.hip): A lane l: row l & 15, logical K 16 (l >> 4) ..
+ 15 as 4 quads x 2 kept values (ascending positions), index nibble = pos0 | pos1 << 2; B lane
l: column l & 15, logical K 8 g + e (e < 8) and 32 + 8 g + e - 8 (e >= 8), g = l >> 4."""
import numpy as np

rs = np.random.RandomState(3)
UP, O, C, H = 18, 32, 32, 40          # pooled dP1 map, its channels, dX channels, dX size
dP = rs.normal(size=(UP, UP, O))
code = rs.randint(0, 4, size=(UP, UP, O))
code[rs.rand(UP, UP, O) < 0.2] = 255
W1 = rs.normal(size=(5, 5, C, O))     # HWIO: conv1 in = 32 (c), out = 32 (o)

# dense reference: dYu (36x36) un-pooled, dX = full correlation with the flipped kernel
dYu = np.zeros((36, 36, O))
for py in range(UP):
    for px in range(UP):
        for o in range(O):
            k = code[py, px, o]
            if k != 255:
                dYu[2 * py + (k >> 1), 2 * px + (k & 1), o] = dP[py, px, o]
pad = np.zeros((44, 44, O))
pad[4:40, 4:40] = dYu
ref = np.zeros((H, H, C))
for a in range(5):
    for b in range(5):
        ref += np.einsum('yxo,co->yxc', pad[a:a + 40, b:b + 40], W1[4 - a, 4 - b])


def mv(r, w, o):                      # masked window value: dYu row r, window w, channel o
    if not (0 <= r < 36 and 0 <= w < UP):
        return 0.0
    k = code[r >> 1, w, o]
    return dP[r >> 1, w, o] if k != 255 and (k >> 1) == (r & 1) else 0.0


def col(r, w, o):
    if not (0 <= r < 36 and 0 <= w < UP):
        return 0
    return int(code[r >> 1, w, o] & 1)


def bweight(eps, kh, t, K, c):
    """B element (logical K of k-step (kh, t), column c) for parity eps."""
    q, p = K >> 2, K & 3
    if t < 2:                          # full quads: quad q = channel 16 t + q, position p = tap kw - eps
        o, kw = 16 * t + q, p + eps
        return W1[4 - kh, 4 - kw, c, o]
    o, cl = 2 * q + (p >> 1), p & 1    # singles: channel pair (2q, 2q+1), pixel column cl
    if eps == 0:
        return W1[4 - kh, 0, c, o] if cl == 0 else 0.0   # tap kw = 4 reads window j, column 0
    return W1[4 - kh, 4, c, o] if cl == 1 else 0.0      # tap kw = 0 reads window j-2, column 1


def smfmac(Avals, Aidx, B):
    """one 16x16x64 sparse product: Avals [64 lanes][8], Aidx [64] (16 bits), B [64 lanes][16]."""
    Ad = np.zeros((16, 64))
    for l in range(64):
        row, g = l & 15, l >> 4
        for qq in range(4):
            nib = (Aidx[l] >> (4 * qq)) & 15
            p0, p1 = nib & 3, nib >> 2
            Ad[row, 16 * g + 4 * qq + p0] += Avals[l][2 * qq]
            Ad[row, 16 * g + 4 * qq + p1] += Avals[l][2 * qq + 1]
    Bd = np.zeros((64, 16))
    for l in range(64):
        n, g = l & 15, l >> 4
        for e in range(16):
            K = 8 * g + e if e < 8 else 32 + 8 * g + (e - 8)
            Bd[K, n] = B[l][e]
    return Ad @ Bd


out = np.zeros((H, H, C))
for y0 in range(0, H, 4):
    for eps in range(2):
        for nt in range(2):
            for jt in range(5):
                acc = np.zeros((16, 16))
                for kh in range(5):
                    for t in range(3):
                        Av, Ai, Bv = [], [], []
                        for l in range(64):
                            m, g = l & 15, l >> 4
                            ry, i = m >> 2, m & 3
                            j = 4 * jt + i
                            r = y0 + ry + kh - 4            # dYu row
                            if t < 2:                        # windows (j - 2 + eps, j - 1 + eps)
                                wa = j - 2 + eps
                                vals, idx = [], 0
                                for qq in range(4):
                                    o = 16 * t + 4 * g + qq
                                    vals += [mv(r, wa, o), mv(r, wa + 1, o)]
                                    idx |= (col(r, wa, o) | (2 + col(r, wa + 1, o)) << 2) << (4 * qq)
                            else:                            # window j (eps 0) / j - 2 (eps 1)
                                ws = j if eps == 0 else j - 2
                                vals, idx = [], 0
                                for qq in range(4):
                                    o = 8 * g + 2 * qq
                                    vals += [mv(r, ws, o), mv(r, ws, o + 1)]
                                    idx |= (col(r, ws, o) | (2 + col(r, ws, o + 1)) << 2) << (4 * qq)
                            Av.append(vals)
                            Ai.append(idx)
                            n = l & 15
                            Bv.append([bweight(eps, kh, t, 8 * g + e if e < 8 else 32 + 8 * g + e - 8, 16 * nt + n)
                                       for e in range(16)])
                        acc += smfmac(Av, Ai, Bv)
                for m in range(16):
                    ry, i = m >> 2, m & 3
                    out[y0 + ry, 2 * (4 * jt + i) + eps, 16 * nt:16 * nt + 16] = acc[m]
print("max |sparse - dense| =", np.abs(out - ref).max(), " max |ref| =", np.abs(ref).max())
assert np.allclose(out, ref, atol=1e-9)
