"""Frozen algorithmic work per Ed25519 verification, for the roofline in bench.py.

Derived ONCE from the reference algorithm (libsodium 1.0.18 crypto_sign_open, ref10 formulas,
which the reference reaches via stp_core/crypto/nacl_wrappers.py:108), NOT from this build's
kernels, so a cleverer kernel gets credit and a wasteful one does not.

Unit: one 32x32->64 multiply-accumulate (MAC) of the radix-2^25.5 schoolbook product, i.e. one
v_mad_u64_u32. A field multiplication is 100 MACs, a squaring 55 (symmetric terms folded).

libsodium's verify, per signature (expected values at random scalars):
  decompression of A (ge25519_frombytes_negate_vartime): 4 S + 9 M around fe25519_pow22523
      (249 S + 11 M)                                                   -> 253 S + 20 M
  table of odd multiples A, 3A, ..., 15A (ge25519_double_scalarmult_vartime):
      1 doubling (4 S + 4 M) + 7 additions (4 M add + 4 M p1p1->p3 + 1 M 2dT)  -> 4 S + 67 M
  main loop, 253 doublings (ge25519_p2_dbl: 4 S, then p1p1->p2: 3 M) and, with width-5 sliding
      windows on both 253-bit scalars, 2 * 256/6 = 85.3 additions, each costing ge25519_add/madd
      (4 M) + p1p1->p3 instead of ->p2 (+1 M) + p1p1->p2 after it (3 M)  -> 1012 S + 759 M + 85.3 * 8 M
  encoding (ge25519_tobytes): fe25519_invert (254 S + 11 M) + 2 M      -> 254 S + 13 M
SHA-512 (3 compressions at the 299-byte template) and the scalar reduction add < 5 % and are
not counted.
"""
MAC_PER_MUL = 100
MAC_PER_SQ = 55

_S_DECOMP, _M_DECOMP = 253, 20
_S_TABLE, _M_TABLE = 4, 67
_ADDS = 2 * 256 / 6
_S_LOOP, _M_LOOP = 253 * 4, 253 * 3 + _ADDS * 8
_S_ENC, _M_ENC = 254, 13


def _mac(s, m):
    return MAC_PER_SQ * s + MAC_PER_MUL * m


# per verification
MAC_DECOMPRESS = _mac(_S_DECOMP, _M_DECOMP)
MAC_TABLE = _mac(_S_TABLE, _M_TABLE)
MAC_LOOP = _mac(_S_LOOP, _M_LOOP)
MAC_ENCODE = _mac(_S_ENC, _M_ENC)
MAC_PER_VERIFY = MAC_DECOMPRESS + MAC_TABLE + MAC_LOOP + MAC_ENCODE
# The Straus path's dominant kernel (pv_msm_kernel) runs the loop over k only: [S]B comes from the
# wide fixed-base comb in pv_straus_b_kernel (PV_STRAUS_WIDE_B) and is added once at the end. Its
# algorithmic work is libsodium's loop without the B-scalar half of the sliding-window additions:
# 253 doublings + 42.7 additions; the encoding runs in pv_encode_kernel.
MAC_MSM_KERNEL = _mac(_S_LOOP, 253 * 3 + _ADDS / 2 * 8)
# The built Straus kernel runs the half-size form of the same check (indy-plenum_amd/csrc/sc25519.h
# sc_halfsize): k = k1 / k2 (mod 8L) with |k1|, k2 < 2^128, so Q' = [k1](+-A) + [k2](-R') over 32
# regular radix-16 windows of both scalars -- 31 x 4 doublings (4 S + 3 M; the last of each window to
# extended, +1 M), per window one cached addition to extended (4 M + 4 M) and one to projective (4 M +
# 3 M) -- then + [k2 S]B (1 M cached form + 4 M + 4 M) and + R' (4 M + 3 M; +1 M for the window's
# output to extended). Its roofline uses this count (the wave-uniform window count actually executed,
# ~33.9 on average at random scalars, is inefficiency against it). A different algorithm than
# MAC_MSM_KERNEL's, counted the same way.
MAC_MSM_HALF_KERNEL = _mac(124 * 4, 124 * 3 + 31 + 32 * 15 + 17)

# The keyed comb path (indy-plenum_amd/csrc/comb.h) performs a DIFFERENT algorithm for the same
# verdict: per request 32 cached-form additions of radix-256 T_A entries (4 M + 4 M to extended) and
# [S]B from the radix-2^24 wide fixed-base comb (11 positions: the top entry converted to extended,
# 2 M, then 10 affine-niels additions, 3 M + 4 M), the last T_A addition to projective (3 M): no
# doublings. Its kernel's roofline uses its own algorithmic work, counted the same way:
MAC_COMB_MSM = MAC_PER_MUL * (32 * 8 + 10 * 7 + 2 - 1)
# it runs as two kernels: pv_comb_b_kernel ([S]B) overlapped with the per-key table build, then
# pv_comb_a_kernel (the 32 T_A additions, the MSM stage and the roofline kernel)
MAC_COMB_B_KERNEL = MAC_PER_MUL * (10 * 7 + 2)
MAC_COMB_MSM_KERNEL = MAC_PER_MUL * (32 * 8 - 1)
# the fused build (PV_BUILD_COMB_FUSED, round 4): pv_comb_ab_kernel runs both halves, [S]B's 10 niels
# additions and the 32 T_A additions, so its algorithmic work is the whole per-request comb count
MAC_COMB_AB_KERNEL = MAC_COMB_MSM
# per distinct key (amortised over the requests that share it): decompression + 31 x 8 doublings
# (4 S + 3 M, the last of each 8 to extended: +1 M) + 32 x 129 table entries (8 M + 1 M each)
MAC_COMB_PER_KEY = _mac(_S_DECOMP, _M_DECOMP) + _mac(31 * 8 * 4, 31 * (8 * 3 + 1)) + MAC_PER_MUL * 32 * 129 * 9

# Peak: v_mad_u64_u32 issues once per 4 cycles per wave64 on a SIMD (measured ~5.2 "cycles at
# 2.4 GHz" under launch overhead and DVFS in profiles/r01_isa_rates.jsonl, and exactly 2x the
# full-rate v_add_u32 time there); 256 CU x 4 SIMD x 64 lanes / 4 cycles x 2.4 GHz.
CUS, SIMDS, LANES, CLOCK_HZ, MAD64_CYCLES = 256, 4, 64, 2.4e9, 4
PEAK_MAC_PER_S = CUS * SIMDS * LANES * CLOCK_HZ / MAD64_CYCLES  # 3.93e13
# What a pure stream of independent v_mad_u64_u32 actually sustains on the chip (clock under load,
# issue): profiles/r01_isa_rates_full.jsonl, 4 waves/SIMD = 4.987e11 wave-instructions/s x 64 lanes.
# Reported beside the nominal peak, never in place of it.
MEASURED_MAD_STREAM_MAC_PER_S = 4.987e11 * 64  # 3.19e13

# Bytes a verification needs from HBM at minimum: the record (64 B signature + ~299 B message)
# + 32 B key + 8 B offset; the verdict bit is negligible.
ALGO_BYTES_PER_VERIFY = 64 + 299 + 32 + 8
HBM_PEAK_BPS = 8.0e12

if __name__ == "__main__":
    print({"MAC_PER_VERIFY": MAC_PER_VERIFY, "MAC_MSM_KERNEL": MAC_MSM_KERNEL, "PEAK_MAC_PER_S": PEAK_MAC_PER_S})
