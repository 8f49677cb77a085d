"""Exhaustive LDS bank-conflict check of the pp3 and MX-fp8 GEMMs' fragment reads
(vtd_gemm_pp3.hip): 64-B group rows, 16-B chunk c of row r stored at position
c ^ (((r >> 3) & 1) << 1).  A ds_read_b128 is serviced in four 16-lane groups
(MI355X_MICROARCH.md, LDS table); a group is conflict-free iff its 16 lanes hit 16
distinct 16-B slots of the 256-B bank row.  Checks the plain A-fragment reads (rows
R0 + fr, chunk fg) and the permuted B-fragment reads of the transposed-accumulator
layout (rows R0 + 8 (fr >> 2) + 4 j + (fr & 3)).  Exit status 0 = conflict-free."""
import sys

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def pos(row, chunk):
    return chunk ^ (((row >> 3) & 1) << 1)


def conflict_free(rows_of):
    for g in GROUPS:
        slots = {(rows_of(l & 15) % 4) * 4 + pos(rows_of(l & 15), l >> 4) for l in g}
        if len(slots) != 16:
            return False
    return True


def mx_pos(row, chunk):
    """MX-fp8 GEMM (vtd_gemm.hip gemm_mx8_kernel): 128-B rows, chunk c at c ^ (row & 7);
    a lane reads chunks fg and fg + 4 of row R0 + fr."""
    return chunk ^ (row & 7)


def mx_conflict_free():
    for r0 in range(0, 256, 16):
        for h in (0, 1):
            for g in GROUPS:
                slots = {((r0 + (l & 15)) * 8 + mx_pos(r0 + (l & 15), (l >> 4) + 4 * h)) % 16
                         for l in g}
                if len(slots) != 16:
                    return False
    return True


def main():
    ok = mx_conflict_free()
    for r0 in range(0, 256, 16):
        ok &= conflict_free(lambda fr, r0=r0: r0 + fr)
    for r0 in range(0, 256, 32):
        for j in (0, 1):
            ok &= conflict_free(lambda fr, r0=r0, j=j: r0 + 8 * (fr >> 2) + 4 * j + (fr & 3))
    print("conflict-free" if ok else "CONFLICT")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
