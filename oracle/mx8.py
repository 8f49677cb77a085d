"""CPU restatement of the MX-fp8 operand format of the VTD_FP8 mode (test infrastructure:
imported only by tests/, never by the product path).

The reference is fp32 Keras (vtd.py); its "fp8 weights on CDNA4 fp8 MFMA" configuration
 has no reference implementation at all, so this module pins the
*format* the build chose: the OCP Microscaling (MX) FP8 layout that gfx950's
block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) consumes:
  - elements: OCP e4m3 ("e4m3fn": bias 7, no infinities, max 448, subnormal quantum 2^-9),
    round-to-nearest-even (gfx950 v_cvt_pk_fp8_f32);
  - one E8M0 scale per 32 consecutive K elements: byte e means 2^(e - 127).
Block scale rule (vtd_mx8.hip): the least power of two 2^E with amax <= 448 * 2^E,
E clamped to [-126, 126] (E = -126 for an all-zero block).
Scale layout: s[k // 128][row][4] (the four 32-blocks of one 128-wide K-step of a row
form one dword).  Parity unpinned against any reference output (none exists); the GPU
tests check the device quantizer against this restatement element for element and the
MX GEMM against the fp64 product of the dequantized operands.
"""
import numpy as np

E4M3_MAX = 448.0


def block_exponent(amax):
    """E = least integer with amax <= 448 * 2^E, via frexp (amax = m 2^ex, m in
    [0.5, 1)): E = ex - 9 + (m > 0.875); clamped to [-126, 126]."""
    amax = np.asarray(amax, dtype=np.float64)
    m, ex = np.frexp(amax)
    e = ex.astype(np.int64) - 9 + (m > 0.875)
    e = np.where(amax > 0, e, -126)
    # float32 subnormal block maxima: the kernel reads the exponent field (0) -> -126
    e = np.where(amax < np.float64(np.finfo(np.float32).tiny), -126, e)
    return np.clip(e, -126, 126)


def round_e4m3(v):
    """Round float64 values with |v| <= 448 to the nearest e4m3 value (ties to even)."""
    v = np.asarray(v, dtype=np.float64)
    a = np.abs(v)
    with np.errstate(divide="ignore"):
        e = np.floor(np.log2(np.where(a > 0, a, 1.0)))
    e = np.maximum(e, -6.0)                     # subnormals share the 2^-6 binade's quantum
    quantum = np.exp2(e - 3.0)
    r = np.rint(a / quantum) * quantum          # np.rint: half to even
    return np.sign(v) * r


def decode_e4m3(b):
    """uint8 e4m3 bytes -> float64 values (0x7f / 0xff = NaN)."""
    b = np.asarray(b, dtype=np.uint8).astype(np.int64)
    s = np.where(b >> 7, -1.0, 1.0)
    E = (b >> 3) & 15
    m = b & 7
    val = np.where(E == 0, m * 2.0 ** -9, (1.0 + m / 8.0) * np.exp2(E - 7.0))
    val = np.where((E == 15) & (m == 7), np.nan, val)
    return s * val


def quantize(x, Kq=None):
    """x [rows][K] (float) -> (values [rows][Kq] float64 = the e4m3 elements, exponents
    [rows][Kq // 32] int) such that x ~= values * 2^E per 32-block."""
    x = np.asarray(x, dtype=np.float64)
    rows, K = x.shape
    Kq = Kq or -(-K // 128) * 128
    xp = np.zeros((rows, Kq))
    xp[:, :K] = x
    blocks = xp.reshape(rows, Kq // 32, 32)
    E = block_exponent(np.abs(blocks).max(axis=2))
    vals = round_e4m3(blocks * np.exp2(-E)[..., None])
    return vals.reshape(rows, Kq), E


def dequantize(q_bytes, s_bytes, rows, Kq):
    """Device buffers -> float64: q [rows][>= Kq] e4m3 bytes, s [Kq // 128][s_rows][4]."""
    q = decode_e4m3(np.asarray(q_bytes)[:rows, :Kq])
    s = np.asarray(s_bytes).reshape(Kq // 128, -1, 4)[:, :rows, :]     # [kstep][row][4]
    e = s.transpose(1, 0, 2).reshape(rows, Kq // 32).astype(np.int64) - 127
    return (q.reshape(rows, Kq // 32, 32) * np.exp2(e)[..., None]).reshape(rows, Kq)
