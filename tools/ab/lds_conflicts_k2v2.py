"""Bank-conflict model of the CURRENT K2 overlap-save passes in complex double (k2_fft_job with
its palindromic power-of-two plans, k2_fft_job_mix for 2560 = 16 x 10 x 16), gfx950 rules of
tools/ab/lds_conflicts64.py.  Addresses are generated exactly as sh_load/sh_store (power-of-two)
and shg_load/shg_store (mixed radix) in rsp_kernels.hip compute them.
usage: lds_conflicts_k2v2.py [SH [rows]]      (prints per pass: reads / writes / twiddle-read cost factor,
1.0 = conflict-free, and the LDS cycles per row weighted by instruction count)"""
import sys
sys.path.insert(0, __file__.rsplit('/', 1)[0])
from lds_conflicts64 import RGROUPS, WGROUPS, gcost  # noqa: E402

NTHR = 256
PTS = 4096


def lidx(i, sh):
    return i + (i >> sh) if sh else i


def tw_row(R):   # compact rows
    return (R - 1).bit_length()


def model(M, rad, sh, pow2):
    rows = PTS // M
    rs = M + (M >> sh)
    Ns = 1
    out = []
    tot_cyc = tot_ideal = 0
    for q, R in enumerate(rad):
        nb = M // R
        total = nb * rows
        NB = -(-total // NTHR)
        rc = wc = tc = ri = wi = ti = 0
        for w0 in range(0, NTHR, 64):
            for t in range(NB):
                betas = [w0 + l + t * NTHR for l in range(64)]
                act = [b for b in betas if b < total]
                if not act:
                    continue
                betas = [b if b < total else act[0] for b in betas]
                rdr = [[] for _ in range(R)]
                wrr = [[] for _ in range(R)]
                twr = [[] for _ in range(tw_row(R))]
                for beta in betas:
                    if pow2:
                        row, j = beta // nb, beta % nb
                        k = j % Ns
                        base = row * rs + lidx(j, sh)
                        for r in range(R):
                            rdr[r].append(base + r * nb + ((r * nb) >> sh))
                        idxD = (j // Ns) * (Ns * R) + k
                        wb = row * rs + lidx(idxD, sh)
                        for r in range(R):
                            wrr[r].append(wb + r * Ns + ((r * Ns) >> sh))
                    else:
                        row, j = beta // nb, beta % nb
                        k = j % Ns
                        for r in range(R):
                            rdr[r].append(row * rs + lidx(j + r * nb, sh))
                        idxD = (j // Ns) * (Ns * R) + k
                        for r in range(R):
                            wrr[r].append(row * rs + lidx(idxD + r * Ns, sh))
                    for i in range(tw_row(R)):
                        twr[i].append(i * Ns + k if COLMAJOR else k * tw_row(R) + i)
                for r in range(R):
                    rc += gcost(rdr[r], RGROUPS, 64); ri += 4
                    wc += gcost(wrr[r], WGROUPS, 32); wi += 8
                if Ns > 1:
                    for i in range(len(twr)):
                        tc += gcost(twr[i], RGROUPS, 64); ti += 4
        out.append((q, R, Ns, rc / ri, wc / wi, (tc / ti) if ti else 0.0, rc + wc + tc, ri + wi + ti))
        tot_cyc += rc + wc + tc
        tot_ideal += ri + wi + ti
        Ns *= R
    return out, tot_cyc, tot_ideal, rows


sh = int(sys.argv[1]) if len(sys.argv) > 1 else 5
COLMAJOR = not (len(sys.argv) > 2 and sys.argv[2] == 'rows')   # compact twiddle layout: [i][k] (current) or [k][i]
for M, rad, pow2 in [(1024, [16, 4, 16], True), (2048, [16, 8, 16], True), (2560, [16, 10, 16], False)]:
    out, c, i, rows = model(M, rad, sh, pow2)
    print('M=%d rows/wg=%d SH=%d  one FFT: %d LDS cycles (conflict-free %d, x%.2f) per workgroup' % (M, rows, sh, c, i, c / i))
    for q, R, Ns, r, w, t, cc, ii in out:
        print('   pass %d R=%2d Ns=%4d  read x%.2f  write x%.2f  tw x%.2f' % (q, R, Ns, r, w, t))
