"""Analytic v_mfma_f64_16x16x4 count of K3's chol_step_pair launches (the MFMA
instructions csrc/chol.hip issues per step j; see the per-phase comments there), for
the cross-check of the PMC MFMA counters (tools/pmc_summary.py: f64_mfma_count,
mfma_busy_cycles_per_f64_mfma; a 16x16x4 f64 MFMA keeps the pipe 64 cycles).
Usage: python tools/k3_mfma_count.py [M] [batch]"""
import json
import sys

LOOKAHEAD = 160 + 64 + 200        # P = W D^T (lower D), column block 0 of P P^T, factor_diag_tile
PAIR_P = 160                      # P_i, split over the two groups
UPD, DIAG, FWD, FWD_DIAG = 160 + 256, 160, 160 + 256, 160


def step_pair_mfmas(nb, j):
    n = LOOKAHEAD
    for i in range(j + 1, nb):
        nt = j + 1 if i == j + 1 else i + 1
        nupd = 0 if i == j + 1 else i - j
        n += PAIR_P * ((nt + 1) // 2)
        for e in range(nt):
            if e < nupd:
                n += DIAG if j + 1 + e == i else UPD
            else:
                n += FWD if e - nupd < j else FWD_DIAG
    return n


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    nb = -(-M // 64)
    per = [batch * step_pair_mfmas(nb, j) for j in range(nb - 1)]
    print(json.dumps({"M": M, "batch": batch, "launches": len(per), "per_launch": per,
                      "avg_per_launch": sum(per) / len(per), "busy_cycles_avg": 64 * sum(per) / len(per)}))


if __name__ == "__main__":
    main()
