"""Exhaustive LDS bank-conflict check of the 256-tile GEMMs' fragment reads (vtd_gemm_w4.hip,
vtd_gemm.hip pp2 / MX-fp8): 128-B LDS rows, 16-B chunk c of row r stored at position
  A image (and every MX / pp2 non-transposed read): c ^ (r & 7)
  B image of the transposed-accumulator layout:     c ^ (r & 7) ^ ((r >> 2) & 4)
A ds_read_b128 is serviced in four 16-lane groups (MI355X_MICROARCH.md, LDS table); a group
is conflict-free iff its 16 lanes hit 16 distinct 16-B slots of the 256-B bank row.
Lane l = (fr = l & 15, fg = l >> 4) reads chunk 4 h + fg (K-half h) of
  plain rows     R0 + fr                               (A fragments, MX operands)
  permuted rows  R0 + 8 (fr >> 2) + 4 jj + (fr & 3)    (B fragments: a lane's accumulators
                                                         are 8 contiguous output columns)
for every wave / block offset R0 the kernels use.  Exit status 0 = conflict-free."""
import sys

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def pos_a(r, c):
    return c ^ (r & 7)


def pos_b(r, c):
    return c ^ (r & 7) ^ ((r >> 2) & 4)


def conflict_free(rows_of, pos, h):
    for g in GROUPS:
        slots = {((rows_of(l & 15) & 1) * 8 + pos(rows_of(l & 15), 4 * h + (l >> 4))) for l in g}
        if len(slots) != 16:
            return False
    return True


def main():
    ok = True
    for h in (0, 1):
        for r0 in range(0, 256, 16):
            ok &= conflict_free(lambda fr, r0=r0: r0 + fr, pos_a, h)
        for r0 in range(0, 256, 32):
            for jj in (0, 1):
                ok &= conflict_free(lambda fr, r0=r0, jj=jj: r0 + 8 * (fr >> 2) + 4 * jj + (fr & 3),
                                    pos_b, h)
        # the permuted rows under the plain swizzle DO conflict (why pos_b exists)
        bad = not conflict_free(lambda fr: 8 * (fr >> 2) + (fr & 3), pos_a, h)
        ok &= bad
    print("conflict-free" if ok else "CONFLICT")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
