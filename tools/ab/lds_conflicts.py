"""Bank-conflict model of the Stockham LDS passes (gfx950 rules, MI355X_MICROARCH.md §LDS):
ds_read_b64 / ds_write_b64 are serviced per 32-lane half-wave, bank = (dword addr) mod 64,
an 8-byte access occupies banks a/4 and a/4+1.  Cost of one instruction = max over banks
of the number of distinct dword addresses mapped to it (1 = conflict-free).
"""
import itertools
import sys


def cost(addrs_c):   # complex index per lane (8 bytes each)
    worst = 0
    for half in (addrs_c[:32], addrs_c[32:]):
        banks = {}
        for a in half:
            for dw in (2 * a, 2 * a + 1):
                banks.setdefault(dw % 64, set()).add(dw)
        worst = max(worst, max(len(s) for s in banks.values()))
    return worst


def radices(m):
    out = []
    while m > 0:
        p = 3 if m == 5 else (4 if m >= 4 else m)
        out.append(1 << p)
        m -= p
    return out


def passes(L, nrows, nthr, rs, pad):
    lg = L.bit_length() - 1
    lidx = (lambda i: i + (i >> 4)) if pad else (lambda i: i)
    Ns = 1
    tot_r = tot_w = n_r = 0
    report = []
    for R in radices(lg):
        nb = L // R
        total = nb * nrows
        rc = wc = cnt = 0
        for w0 in range(0, nthr, 64):
            for t in range((total + nthr - 1) // nthr):
                lanes = [w0 + l + t * nthr for l in range(64)]
                lanes = [b for b in lanes if b < total]
                if len(lanes) < 64:
                    lanes += [lanes[-1]] * (64 - len(lanes))
                for r in range(R):
                    ra, wa = [], []
                    for beta in lanes:
                        row, j = divmod(beta, nb)
                        k = j % Ns
                        ra.append(row * rs + lidx(j + r * nb))
                        idxD = (j // Ns) * Ns * R + k
                        wa.append(row * rs + lidx(idxD + r * Ns))
                    rc += cost(ra); wc += cost(wa); cnt += 1
        report.append((R, Ns, rc / cnt, wc / cnt))
        Ns *= R
    return report


if __name__ == '__main__':
    for name, L, nrows, nthr, rs, pad in [
            ('K1 P128 B8 NT8 Ppad132', 128, 64, 512, 132, False),
            ('K1 P128 pad16 rs=136+4', 128, 64, 512, 140, True),
            ('K1 P128 pad16 rs=136', 128, 64, 512, 136, True),
            ('K2 M2048 rows2 rs2176', 2048, 2, 256, 2176, True),
            ('K2 M1024 rows4 rs1088', 1024, 4, 256, 1088, True),
            ('K2 M2048 nopad rs2048+4', 2048, 2, 256, 2052, False)]:
        print(name)
        for R, Ns, rc, wc in passes(L, nrows, nthr, rs, pad):
            print('   R=%2d Ns=%4d  read x%.2f  write x%.2f' % (R, Ns, rc, wc))
