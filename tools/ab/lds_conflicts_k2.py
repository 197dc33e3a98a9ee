"""Bank-conflict model of the K2 overlap-save passes (k2_block, radix plans k2_rad in
rsp_internal.h) for complex-double elements, gfx950 rules as tools/ab/lds_conflicts64.py.
usage: lds_conflicts_k2.py [SH ...]   (prints read / write cost factors per pass; 1.0 = conflict-free)
"""
import sys
sys.path.insert(0, __file__.rsplit('/', 1)[0])
from lds_conflicts64 import RGROUPS, WGROUPS, gcost  # noqa: E402


def k2_plan(M):
    if M == 2560:
        return [8, 8, 8, 5]
    m = M.bit_length() - 1
    n3, rm = divmod(m, 3)
    if rm == 0:
        return [8] * n3
    if rm == 2:
        return [8] * n3 + [4]
    return [8] * (n3 - 1) + [4, 4]


def passes(M, rows, nthr, sh, rad):
    rs = M + (M >> sh if sh else 0)
    lidx = (lambda i: i + (i >> sh)) if sh else (lambda i: i)
    Ns = 1
    rep = []
    for R in rad:
        nb = M // R
        total = nb * rows
        NB = -(-total // nthr)
        rc = wc = cnt = 0
        for w0 in range(0, nthr, 64):
            for t in range(NB):
                lanes = [w0 + l + t * nthr for l in range(64)]
                if lanes[0] >= total:
                    continue
                lanes = [b if b < total else lanes[0] for b in lanes]
                for r in range(R):
                    ra, wa = [], []
                    for beta in lanes:
                        row, j = divmod(beta, nb)
                        ra.append(row * rs + lidx(j + r * nb))
                        idxD = (j // Ns) * Ns * R + j % Ns
                        wa.append(row * rs + lidx(idxD + r * Ns))
                    rc += gcost(ra, RGROUPS, 64) / 4.0
                    wc += gcost(wa, WGROUPS, 32) / 8.0
                    cnt += 1
        rep.append((R, Ns, rc / cnt, wc / cnt, cnt))
        Ns *= R
    return rep


if __name__ == '__main__':
    shs = [int(x) for x in sys.argv[1:]] or [0, 2, 3, 4, 5]
    for sh in shs:
        tot = 0.0
        for M, rows in [(2560, 1), (1024, 2)]:
            for inv in (False, True):
                rad = k2_plan(M)[::-1] if inv else k2_plan(M)
                rep = passes(M, rows, 320, sh, rad)
                print('SH=%d M=%d %s: ' % (sh, M, 'inv' if inv else 'fwd') +
                      '  '.join('R%d/Ns%d r%.2f w%.2f' % (R, Ns, rc, wc) for R, Ns, rc, wc, _ in rep))
                tot += sum((rc * 4 + wc * 13) * n for R, Ns, rc, wc, n in rep) * (M // 2560 if M == 2560 else 1)
        print('SH=%d weighted LDS cycles %.0f' % (sh, tot))
