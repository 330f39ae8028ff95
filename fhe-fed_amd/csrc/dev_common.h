// dev_common.h — device helpers shared by the gfx950 kernel files (kernels.hip,
// keyswitch.hip): 64-bit modular arithmetic (Shoup, lazy butterflies, borrow-free
// reductions), complex f64 helpers and the ChaCha20 / Gaussian / ternary samplers.
#pragma once

#include <hip/hip_runtime.h>

#include "shelfi_internal.h"

namespace shelfi {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------ modular ops ----
__device__ __forceinline__ uint64_t addmod(uint64_t a, uint64_t b, uint64_t q) {
  uint64_t s = a + b;
  return s >= q ? s - q : s;
}
__device__ __forceinline__ uint64_t submod(uint64_t a, uint64_t b, uint64_t q) {
  return a >= b ? a - b : a + q - b;
}
// x * w mod q, w < q, w' = floor(w 2^64 / q), any 64-bit x.
__device__ __forceinline__ uint64_t shoup_mul(uint64_t x, uint64_t w, uint64_t wp, uint64_t q) {
  uint64_t hi = __umul64hi(x, wp);
  uint64_t r = x * w - hi * q;
  return r >= q ? r - q : r;
}
// x mod q for any 64-bit x (Shoup with w = 1).
__device__ __forceinline__ uint64_t red64(uint64_t x, uint64_t q, uint64_t one_sh) {
  uint64_t hi = __umul64hi(x, one_sh);
  uint64_t r = x - hi * q;
  return r >= q ? r - q : r;
}
// ---- lazy NTT arithmetic (bit-exact after the final canonicalisation) -----
// High 64 bits of x*y from three 32x32 partial products, all carries out of the low
// 64 bits dropped (x0*y0 and the sum of the middle low halves): the exact value minus
// 0, 1 or 2.  Six VALU ops (three quarter-rate) instead of eight for the carried form.
__device__ __forceinline__ uint64_t umulhi_approx(uint64_t x, uint64_t y) {
  const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32), y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32);
  return (uint64_t)x1 * y1 + (((uint64_t)x1 * y0) >> 32) + (((uint64_t)x0 * y1) >> 32);
}
// x * w mod q up to 3 extra q: result in [0, 4q) for any 64-bit x (Shoup with the
// quotient short by at most 2).  x*w - h*q is formed as x*w + h*(2^64 - q) so the
// second 64-bit product takes the first as its v_mad_u64_u32 addend (no borrow chain).
__device__ __forceinline__ uint64_t shoup_lazy(uint64_t x, uint64_t w, uint64_t wp, uint64_t q) {
  const uint64_t h = umulhi_approx(x, wp), nq = (uint64_t)0 - q;
  const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32), w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
  const uint32_t h0 = (uint32_t)h, h1 = (uint32_t)(h >> 32), n0 = (uint32_t)nq, n1 = (uint32_t)(nq >> 32);
  const uint64_t lo = (uint64_t)h0 * n0 + (uint64_t)x0 * w0;  // mod 2^64
  // the cross terms only touch the high word: one v_add3_u32 there (left to itself the
  // compiler zero-extends them and spends a v_mov + 64-bit add)
  const uint32_t c1 = x1 * w0 + x0 * w1, c2 = h1 * n0 + h0 * n1;
  uint32_t hi;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(lo >> 32)), "v"(c1), "v"(c2));
  return ((uint64_t)hi << 32) | (uint32_t)lo;
}
// a + (x * w mod q up to 3 extra q), for a + 4q < 2^64: the addend rides in the first
// v_mad_u64_u32 (x0 w0 + a), so the forward butterfly's X = x + t costs nothing extra.
__device__ __forceinline__ uint64_t shoup_lazy_add(uint64_t x, uint64_t w, uint64_t wp, uint64_t q, uint64_t a) {
  const uint64_t h = umulhi_approx(x, wp), nq = (uint64_t)0 - q;
  const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32), w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
  const uint32_t h0 = (uint32_t)h, h1 = (uint32_t)(h >> 32), n0 = (uint32_t)nq, n1 = (uint32_t)(nq >> 32);
  const uint64_t lo = (uint64_t)h0 * n0 + ((uint64_t)x0 * w0 + a);  // mod 2^64
  const uint32_t c1 = x1 * w0 + x0 * w1, c2 = h1 * n0 + h0 * n1;
  uint32_t hi;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(lo >> 32)), "v"(c1), "v"(c2));
  return ((uint64_t)hi << 32) | (uint32_t)lo;
}
// Same bound, as x*w - h*q (the form the inverse butterflies schedule better).
__device__ __forceinline__ uint64_t shoup_lazy_sub(uint64_t x, uint64_t w, uint64_t wp, uint64_t q) {
  return x * w - umulhi_approx(x, wp) * q;
}
// X >= 4q ? X - 4q : X, selected on the subtraction's own borrow.
__device__ __forceinline__ uint64_t sub4q_if_ge(uint64_t X, uint64_t q) {
  uint64_t d;
  const bool borrow = __builtin_sub_overflow(X, q << 2, &d);
  return borrow ? X : d;
}
// Forward (CT) butterfly keeping values in [0, 8q) (q < 2^60, so 8q < 2^63).
__device__ __forceinline__ void ct_bfly(uint64_t& X, uint64_t& Y, uint64_t W, uint64_t Wp,
                                        uint64_t q) {
  const uint64_t x = sub4q_if_ge(X, q);      // [0, 4q)
  const uint64_t t = shoup_lazy(Y, W, Wp, q);  // [0, 4q)
  X = x + t;                                 // [0, 8q)
  Y = x + (q << 2) - t;                      // (0, 8q)
}
// Inverse (GS) butterfly keeping values in [0, 4q).
__device__ __forceinline__ void gs_bfly(uint64_t& X, uint64_t& Y, uint64_t W, uint64_t Wp,
                                        uint64_t q) {
  const uint64_t s = X + Y;                  // [0, 8q)
  const uint64_t d = X + (q << 2) - Y;       // (0, 8q)
  X = sub4q_if_ge(s, q);                     // [0, 4q)
  Y = shoup_lazy_sub(d, W, Wp, q);           // [0, 4q)
}
// ---- borrow-free conditional subtraction and one-step reduction ------------
// d = x - c as x + (2^64 - c) (v_lshl_add_u64, no VCC carry chain); when x < c < 2^63
// d wraps to >= 2^63, so its sign selects x (v_bfi_b32 on the sign mask).
// (v_bfi_b32 spelled out: left to itself the compiler rebuilds the select from a 64-bit
// compare + v_cndmask and v_max_i32 + v_and_or_b32, 6 instructions instead of 4.)
__device__ __forceinline__ uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b, bitwise
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint64_t csub_neg(uint64_t x, uint64_t negc) {
  const uint64_t d = x + negc;
  const uint32_t m = (uint32_t)((int32_t)(uint32_t)(d >> 32) >> 31);
  const uint32_t lo = bfi32(m, (uint32_t)x, (uint32_t)d);
  const uint32_t hi = bfi32(m, (uint32_t)(x >> 32), (uint32_t)(d >> 32));
  return ((uint64_t)hi << 32) | lo;
}
// any u64 x -> [0, q) (TowerConst::red_ok, q >= 2^40): quotient estimate from x's high
// word, short by at most 1, then one conditional subtraction.
__device__ __forceinline__ uint64_t red_any(uint64_t x, const TowerConst& c) {
  const uint32_t k = __umulhi((uint32_t)(x >> 32), c.red_r) >> c.red_sh;
  const uint64_t r = x + (uint64_t)k * (uint32_t)c.nq + ((uint64_t)(k * (uint32_t)(c.nq >> 32)) << 32);
  return csub_neg(r, c.nq);
}
// Towers below this bound skip the forward reductions of the encrypt passes (NORED).
constexpr uint64_t kNoRedQ = 1ull << 57;
// Reduction schedule for canonical inputs (bounds in units of q): stage s reduces its x
// inputs only when its outputs could otherwise reach 16q; fwd_bound(S) bounds the
// outputs after S stages.
constexpr bool fwd_red_at(int s) {
  int B = 1;
  for (int i = 0; i < s; ++i) B = (B + 4 > 16 ? 8 : B) + 4;
  return B + 4 > 16;
}
constexpr int fwd_bound(int S) {
  int B = 1;
  for (int i = 0; i < S; ++i) B = (B + 4 > 16 ? 8 : B) + 4;
  return B;
}
// Forward (CT) butterfly with the input reduction scheduled by the caller: inputs
// x < 16q (RED: x -= 8q when x >= 8q, so x < 8q) or x < 12q (no reduction), any y;
// outputs X = x + t, Y = x + 4q - t with t = y w mod q in [0, 4q): below 16q (q < 2^60).
// (Round 4: X = x + t comes out of the product's first multiply-add, and Y = 2x + 4q - X is one
// v_lshl_add_u64 and a 64-bit subtraction -- 3 VALU for the pair instead of 4; the same values,
// Y wraps mod 2^64 only in between: x + 4q - t itself is below 20q.)
template <bool RED>
__device__ __forceinline__ void ct_bfly_s(uint64_t& X, uint64_t& Y, uint64_t W, uint64_t Wp,
                                          uint64_t q, uint64_t n8q) {
  const uint64_t x = RED ? csub_neg(X, n8q) : X;
  const uint64_t s = shoup_lazy_add(Y, W, Wp, q, x);  // x + t
  Y = (x << 1) + (q << 2) - s;                        // x + 4q - t
  X = s;
}

// Inverse (GS) butterfly, [0, 4q) in and out, borrow-free reduction of the sum (the generic
// passes; the compile-time ones schedule the reduction with gs_bfly_b below).
__device__ __forceinline__ void gs_bfly_s(uint64_t& X, uint64_t& Y, uint64_t W, uint64_t Wp,
                                          uint64_t q, uint64_t n4q) {
  const uint64_t x = X, y = Y;
  X = csub_neg(x + y, n4q);
  Y = shoup_lazy(x + (q << 2) - y, W, Wp, q);
}
// Inverse (GS) butterfly with the sum's reduction scheduled by the caller (q < 2^60): inputs
// below B = 4q (B8 false: X = x + y < 8q, left unreduced) or B = 8q (B8: X = x + y < 16q,
// reduced by 8q to < 8q); Y = (x + B - y) w lazily, < 4q.  Inside a register group the bound
// of a stage's inputs is known at compile time: an element written as a sum (X) by the
// previous stage is below 8q, one written as a product (Y) below 4q, so only pairs of sums
// pay the reduction.
template <bool B8>
__device__ __forceinline__ void gs_bfly_b(uint64_t& X, uint64_t& Y, uint64_t W, uint64_t Wp, uint64_t q,
                                          uint64_t n8q) {
  const uint64_t x = X, y = Y;
  X = B8 ? csub_neg(x + y, n8q) : x + y;
  Y = shoup_lazy(x + (q << (B8 ? 3 : 2)) - y, W, Wp, q);
}
// Stage v (pairs 2^v apart) of a register group whose inputs are below 8q (IN8) or 4q: does
// the pair at group index a take the 8q form?
template <bool IN8>
__device__ constexpr bool gs_in8(int v, int a) {
  return v == 0 ? IN8 : ((a >> (v - 1)) & 1) == 0;
}
// [0, 8q) -> [0, q)
__device__ __forceinline__ uint64_t canon8(uint64_t x, uint64_t q) {
  x = x >= 4 * q ? x - 4 * q : x;
  x = x >= 2 * q ? x - 2 * q : x;
  return x >= q ? x - q : x;
}
// [0, 4q) -> [0, q)
__device__ __forceinline__ uint64_t canon4(uint64_t x, uint64_t q) {
  x = x >= 2 * q ? x - 2 * q : x;
  return x >= q ? x - q : x;
}

// a * b mod q for arbitrary a, b < q (no precomputed companion).
__device__ __forceinline__ uint64_t mulmod_generic(uint64_t a, uint64_t b, const TowerConst& c) {
  uint64_t hi = __umul64hi(a, b), lo = a * b;
  return addmod(shoup_mul(hi, c.r64, c.r64_shoup, c.q), red64(lo, c.q, c.one_shoup), c.q);
}
__device__ __forceinline__ uint64_t mod_signed_dev(int64_t v, const TowerConst& c) {
  // one reduction of |v| and a sign fix-up (two branch-free reductions cost registers)
  const bool neg = v < 0;
  const uint64_t r = red64(neg ? (uint64_t)0 - (uint64_t)v : (uint64_t)v, c.q, c.one_shoup);
  return (neg && r) ? c.q - r : r;
}
__device__ __forceinline__ uint64_t small_mod(int64_t v, uint64_t q) {  // |v| < q
  return v < 0 ? q - (uint64_t)(-v) : (uint64_t)v;
}
__device__ __forceinline__ uint32_t bitrev_dev(uint32_t x, uint32_t bits) {
  return bits ? (__brev(x) >> (32 - bits)) : 0;
}
// llround (ties away from zero), the oracle's or_round_half_away.
__device__ __forceinline__ int64_t round_half_away(double x) {
  double t = trunc(x);
  double d = __dsub_rn(x, t);
  if (d >= 0.5) t = __dadd_rn(t, 1.0);
  else if (d <= -0.5) t = __dsub_rn(t, 1.0);
  return (int64_t)t;
}
// complex helpers: (a+bi)(c+di) = (ac - bd, ad + bc), each op rounded (no FMA).
__device__ __forceinline__ double2 cmul(double2 v, double2 w) {
  return make_double2(__dsub_rn(__dmul_rn(v.x, w.x), __dmul_rn(v.y, w.y)),
                      __dadd_rn(__dmul_rn(v.x, w.y), __dmul_rn(v.y, w.x)));
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) {
  return make_double2(__dadd_rn(a.x, b.x), __dadd_rn(a.y, b.y));
}
__device__ __forceinline__ double2 csub(double2 a, double2 b) {
  return make_double2(__dsub_rn(a.x, b.x), __dsub_rn(a.y, b.y));
}

// ---------------------------------------------------------------- ChaCha20 ----
struct Key8 {
  uint32_t k[8];
};
#define CH_QR(a, b, c, d)                      \
  a += b; d ^= a; d = __builtin_rotateleft32(d, 16); \
  c += d; b ^= c; b = __builtin_rotateleft32(b, 12); \
  a += b; d ^= a; d = __builtin_rotateleft32(d, 8);  \
  c += d; b ^= c; b = __builtin_rotateleft32(b, 7);

// RFC 8439 block function with a 64-bit counter (words 12-13) and 64-bit nonce
// (words 14-15); out = 8 u64 words (2i, 2i+1).
__device__ __forceinline__ void chacha20_block(const Key8& key, uint64_t counter, uint64_t nonce,
                                               uint64_t out[8]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key.k[0], key.k[1], key.k[2], key.k[3], key.k[4], key.k[5], key.k[6], key.k[7],
                    (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)nonce,
                    (uint32_t)(nonce >> 32)};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = s[i];
#pragma unroll 2
  for (int i = 0; i < 10; ++i) {
    CH_QR(x[0], x[4], x[8], x[12]);
    CH_QR(x[1], x[5], x[9], x[13]);
    CH_QR(x[2], x[6], x[10], x[14]);
    CH_QR(x[3], x[7], x[11], x[15]);
    CH_QR(x[0], x[5], x[10], x[15]);
    CH_QR(x[1], x[6], x[11], x[12]);
    CH_QR(x[2], x[7], x[8], x[13]);
    CH_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
    out[i] = (uint64_t)(x[2 * i] + s[2 * i]) | ((uint64_t)(x[2 * i + 1] + s[2 * i + 1]) << 32);
}

// The same block as 16 little-endian 32-bit words.
__device__ __forceinline__ void chacha20_block32(const Key8& key, uint64_t counter, uint64_t nonce,
                                                 uint32_t out[16]) {
  uint64_t w[8];
  chacha20_block(key, counter, nonce, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out[2 * i] = (uint32_t)w[i];
    out[2 * i + 1] = (uint32_t)(w[i] >> 32);
  }
}

// One block computed by the 4 lanes of a quad: lane j = lane mod 4 runs column j's quarter
// rounds, and the diagonal rounds rotate rows 1..3 across the quad (DPP quad_perm), as SIMD
// ChaCha implementations rotate vector lanes; a quad transpose at the end hands lane j words
// 4j .. 4j + 3 of the block (the same words chacha20_block32 gives).  A quarter of the
// instructions of chacha20_block32 per lane.  Every lane of the quad must be active and pass
// the same counter and nonce.
template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ void chacha20_quad(const Key8& key, uint64_t counter, uint64_t nonce,
                                              uint32_t out[4]) {
  constexpr int ROT1 = 0x39, ROT2 = 0x4E, ROT3 = 0x93, XOR1 = 0xB1;  // lane j <- lane (j + r) mod 4
  const uint32_t j = threadIdx.x & 3;
  const bool j1 = j & 1, j2 = j & 2;
  const auto pick = [&](uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
    return j2 ? (j1 ? v3 : v2) : (j1 ? v1 : v0);
  };
  const uint32_t sa = pick(0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u);
  const uint32_t sb = pick(key.k[0], key.k[1], key.k[2], key.k[3]);
  const uint32_t sc = pick(key.k[4], key.k[5], key.k[6], key.k[7]);
  const uint32_t sd = pick((uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)nonce, (uint32_t)(nonce >> 32));
  uint32_t a = sa, b = sb, c = sc, d = sd;
#pragma unroll 2
  for (int i = 0; i < 10; ++i) {
    CH_QR(a, b, c, d);  // column j
    b = quad_perm<ROT1>(b);
    c = quad_perm<ROT2>(c);
    d = quad_perm<ROT3>(d);
    CH_QR(a, b, c, d);  // diagonal j: x[j], x[4 + (j+1)%4], x[8 + (j+2)%4], x[12 + (j+3)%4]
    b = quad_perm<ROT3>(b);
    c = quad_perm<ROT2>(c);
    d = quad_perm<ROT1>(d);
  }
  // lane j holds x[j], x[4 + j], x[8 + j], x[12 + j]: transpose the quad's 4 x 4 words
  uint32_t X[4] = {a + sa, b + sb, c + sc, d + sd};
#pragma unroll
  for (int p = 0; p < 2; ++p) {  // swap the off-diagonal 2 x 2 blocks (lanes j ^ 2)
    const uint32_t r = quad_perm<ROT2>(j2 ? X[p] : X[p + 2]);
    if (j2) X[p] = r; else X[p + 2] = r;
  }
#pragma unroll
  for (int p = 0; p < 4; p += 2) {  // transpose each 2 x 2 block (lanes j ^ 1)
    const uint32_t r = quad_perm<XOR1>(j1 ? X[p] : X[p + 1]);
    if (j1) X[p] = r; else X[p + 1] = r;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = X[i];
}

// ---- encrypt sampler v2 (round 3; DESIGN.md §2.3, oracle or_sample_encrypt) ----
// Stream of ciphertext g (nonce (1 << 56) | g), in ChaCha20 blocks of 16 32-bit words, with
// N16 = N / 16 and coefficient j = h + N16 i (h < N16, i < 16):
//   v  : blocks [0, N/64): block h/4, words 4 (h mod 4) .. +3 = a 128-bit U (word 0 lowest);
//        v_j = trit_i - 1 with trit_i the i-th base-3 digit of U / 2^128 (U <- 3U, the carry
//        out of bit 128 is the digit): 16 ternary samples per 128 bits (was one 64-bit word
//        each); the 16-digit pattern is within 3^16 / 2^128 < 2^-102 of uniform.
//   e0 : block N/64 + h, word i;  e1: block N/64 + N16 + h, word i: a 32-bit word w gives the
//        sign (w & 1) and the top 31 bits of a 63-bit uniform U63 = (w >> 1) 2^32 + lo32;
//        |e| = #{t : U63 >= cdt[t]}.  lo32 (word i of block N/64 + 2 N16 + h for e0, + 3 N16
//        for e1) only matters when w >> 1 equals the top 31 bits of a CDT entry (probability
//        ~2^-26 per sample) and is generated only then: the distribution is the 63-bit CDT's.
// The v / e0 / e1 words of a column of 16 coefficients come from 1/4 + 1 + 1 ChaCha blocks
// instead of 6.
__device__ __forceinline__ uint32_t trit_next(uint32_t (&u)[4]) {  // U <- 3U mod 2^128, returns the carry
  uint64_t c = 0;
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    c = (uint64_t)u[l] * 3u + c;
    u[l] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}
// Word i of a stream block, out of line: the rare tie path of gauss32 (kept out of the
// unrolled sampling loops' code).
__device__ __noinline__ uint32_t chacha20_word(Key8 key, uint64_t counter, uint64_t nonce, uint32_t i) {
  uint32_t t[16];
  chacha20_block32(key, counter, nonce, t);
  uint32_t r = t[0];
#pragma unroll
  for (int j = 1; j < 16; ++j) r = (i == (uint32_t)j) ? t[j] : r;
  return r;
}
// |e| and sign from a 32-bit word, tab_hi / tab_lo = the CDT's top 31 / low 32 bits, padded to
// 64 entries with 0xFFFFFFFF tops (above every 31-bit value); lo32() fetches the tie word.
template <class Lo>
__device__ __forceinline__ int64_t gauss32(uint32_t w, const uint32_t* tab_hi, const uint32_t* tab_lo, Lo lo32) {
  const uint32_t H = w >> 1;
  uint32_t k = 0;
#pragma unroll
  for (uint32_t step = 32; step; step >>= 1) k += (tab_hi[k + step - 1] < H) ? step : 0u;
  if (tab_hi[k] == H) {  // tie on the top 31 bits: the low half decides (rare, divergent)
    const uint32_t lo = lo32();
    while (k < 64 && tab_hi[k] == H && tab_lo[k] <= lo) ++k;
  }
  return (w & 1) ? -(int64_t)k : (int64_t)k;
}

__device__ __forceinline__ int64_t gauss_sample(uint64_t r, const uint64_t* __restrict__ cdt,
                                                int T) {
  const uint64_t u = r >> 1;
  int64_t k = 0;
  for (int i = 0; i < T; ++i) k += (u >= cdt[i]) ? 1 : 0;
  return (r & 1) ? -k : k;
}
__device__ __forceinline__ int64_t ternary_sample(uint64_t r) { return (int64_t)(r % 3) - 1; }
// The same count by branch-free binary search over the table padded to 64 entries with
// 2^64 - 1 (never <= a 63-bit u) and staged in LDS: 6 steps instead of T = 43 64-bit
// compares (the table is non-decreasing, so #{i : u >= cdt[i]} is an upper bound).
__device__ __forceinline__ int64_t gauss_sample_lds(uint64_t r, const uint64_t* tab) {
  const uint64_t u = r >> 1;
  uint32_t k = 0;
#pragma unroll
  for (uint32_t step = 32; step; step >>= 1) k += (u >= tab[k + step - 1]) ? step : 0u;
  return (r & 1) ? -(int64_t)k : (int64_t)k;
}

// ---- LDS block passes: radix-2^k register chunks -------------------------
// LDS layout: plain.  An XOR swizzle (i ^ h(i >> 5)) that removes the 8-/4-way bank
// conflicts of the d = 4 / d = 1 chunks measured SLOWER (30.4 vs 27.5 ms for the
// ntt_fwd_blocks share of a 11,424-ciphertext encrypt sweep): this pass is bound by
// VALU issue (64-bit Shoup products), not by LDS.  lds_sw is kept as the one place
// to change the layout.
__device__ __forceinline__ uint32_t lds_sw(uint32_t i) { return i; }
// 16-byte fill/drain: elements (2p, 2p+1) share one aligned 16-byte LDS slot under
// lds_sw, swapped when the XOR flips bit 0.
__device__ __forceinline__ void lds_put2(uint64_t* sm, uint32_t p, ulonglong2 v) {
  const uint32_t i = 2 * p, s = lds_sw(i);
  if (s & 1) {
    const uint64_t t = v.x;
    v.x = v.y;
    v.y = t;
  }
  reinterpret_cast<ulonglong2*>(sm)[s >> 1] = v;
}
__device__ __forceinline__ ulonglong2 lds_get2(const uint64_t* sm, uint32_t p) {
  const uint32_t i = 2 * p, s = lds_sw(i);
  ulonglong2 v = reinterpret_cast<const ulonglong2*>(sm)[s >> 1];
  if (s & 1) {
    const uint64_t t = v.x;
    v.x = v.y;
    v.y = t;
  }
  return v;
}
// A block of blk = 2^blkLog contiguous elements (global block index b) sits in LDS.
// Its stages are taken KCH = 3 at a time: each thread loads a set of 2^KCH elements
// that only interact among themselves during those stages, runs them in registers
// (2^KCH - 1 twiddle pairs), and writes the set back — one barrier per chunk instead
// of one per stage.  256 threads; blocks of 2^blkLog <= 4096 elements (ntt_block_log).
//
// Forward (CT, half-size h = blk/2 .. 1): a chunk of k stages starting at half-size
// h0 works on sets {j0 + d m}, d = h0 / 2^(k-1), j0 = g 2 h0 + off (off < d).
template <int KC>
__device__ __forceinline__ void fwd_chunk(uint64_t* sm, uint32_t blk, uint32_t h0Log, uint32_t b,
                                          uint32_t blkLog, uint32_t logN,
                                          const uint64_t* __restrict__ w,
                                          const uint64_t* __restrict__ wp, uint64_t q) {
  constexpr int M = 1 << KC;
  const uint32_t dLog = h0Log - (KC - 1), d = 1u << dLog;
  const uint32_t nsets = blk >> KC;
  const uint64_t gbase = (uint64_t)b << blkLog;  // global index of the block start
  for (uint32_t set = threadIdx.x; set < nsets; set += 256) {
    const uint32_t g = set >> dLog, off = set & (d - 1);
    const uint32_t j0 = (g << (h0Log + 1)) + off;
    uint64_t x[M];
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = sm[lds_sw(j0 + (m << dLog))];
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const int hm = 1 << (KC - 1 - i);          // half-size in units of d
      const uint32_t hLog = h0Log - i;           // log2 of the half-size
      const uint32_t s = logN - 1 - hLog;        // global stage: m_stage = 2^s
#pragma unroll
      for (int gs = 0; gs < (1 << i); ++gs) {    // 2^i twiddle groups at this stage
        const uint64_t gi = (gbase + j0 + ((uint64_t)(gs * 2 * hm) << dLog)) >> (hLog + 1);
        const uint64_t W = w[(1ull << s) + gi], Wp = wp[(1ull << s) + gi];
#pragma unroll
        for (int mm = 0; mm < hm; ++mm) {
          const int m0 = gs * 2 * hm + mm, m1 = m0 + hm;
          ct_bfly(x[m0], x[m1], W, Wp, q);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) sm[lds_sw(j0 + (m << dLog))] = x[m];
  }
}

// Runs every stage of the block (local half-sizes blk/2 .. 1), chunked 3 at a time.
__device__ __forceinline__ void ntt_fwd_block_stages(uint64_t* sm, uint32_t blkLog, uint32_t b,
                                                     uint32_t logN, const uint64_t* __restrict__ w,
                                                     const uint64_t* __restrict__ wp, uint64_t q) {
  const uint32_t blk = 1u << blkLog;
  uint32_t left = blkLog;  // stages remaining; next half-size = 2^(left-1)
  while (left > 0) {
    const uint32_t h0Log = left - 1;
    if (left >= 3) {
      fwd_chunk<3>(sm, blk, h0Log, b, blkLog, logN, w, wp, q);
      left -= 3;
    } else if (left == 2) {
      fwd_chunk<2>(sm, blk, h0Log, b, blkLog, logN, w, wp, q);
      left -= 2;
    } else {
      fwd_chunk<1>(sm, blk, h0Log, b, blkLog, logN, w, wp, q);
      left -= 1;
    }
    __syncthreads();
  }
}

// Inverse (GS, half-size t = 1 .. blk/2): a chunk of k stages starting at half-size
// t0 works on sets {j0 + t0 m}, j0 = g t0 2^k + off (off < t0); twiddle for half-size
// t at global element j: ipsi_rev[N/(2t) + j/(2t)].
template <int KC>
__device__ __forceinline__ void inv_chunk(uint64_t* sm, uint32_t blk, uint32_t t0Log, uint32_t b,
                                          uint32_t blkLog, uint32_t logN,
                                          const uint64_t* __restrict__ w,
                                          const uint64_t* __restrict__ wp, uint64_t q) {
  constexpr int M = 1 << KC;
  const uint32_t t0 = 1u << t0Log;
  const uint32_t nsets = blk >> KC;
  const uint64_t gbase = (uint64_t)b << blkLog;
  for (uint32_t set = threadIdx.x; set < nsets; set += 256) {
    const uint32_t g = set >> t0Log, off = set & (t0 - 1);
    const uint32_t j0 = (g << (t0Log + KC)) + off;
    uint64_t x[M];
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = sm[lds_sw(j0 + (m << t0Log))];
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const int hm = 1 << i;                  // half-size in units of t0
      const uint32_t tLog = t0Log + i;
      const uint64_t hbase = (uint64_t)1 << (logN - 1 - tLog);  // N / (2t)
#pragma unroll
      for (int gs = 0; gs < (M >> (i + 1)); ++gs) {
        const uint64_t gi = (gbase + j0 + ((uint64_t)(gs * 2 * hm) << t0Log)) >> (tLog + 1);
        const uint64_t W = w[hbase + gi], Wp = wp[hbase + gi];
#pragma unroll
        for (int mm = 0; mm < hm; ++mm) {
          const int m0 = gs * 2 * hm + mm, m1 = m0 + hm;
          gs_bfly(x[m0], x[m1], W, Wp, q);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) sm[lds_sw(j0 + (m << t0Log))] = x[m];
  }
}

__device__ __forceinline__ void ntt_inv_block_stages(uint64_t* sm, uint32_t blkLog, uint32_t b,
                                                     uint32_t logN, const uint64_t* __restrict__ w,
                                                     const uint64_t* __restrict__ wp, uint64_t q) {
  const uint32_t blk = 1u << blkLog;
  uint32_t t0Log = 0;
  while (t0Log < blkLog) {
    const uint32_t left = blkLog - t0Log;
    if (left >= 3) {
      inv_chunk<3>(sm, blk, t0Log, b, blkLog, logN, w, wp, q);
      t0Log += 3;
    } else if (left == 2) {
      inv_chunk<2>(sm, blk, t0Log, b, blkLog, logN, w, wp, q);
      t0Log += 2;
    } else {
      inv_chunk<1>(sm, blk, t0Log, b, blkLog, logN, w, wp, q);
      t0Log += 1;
    }
    __syncthreads();
  }
}

// Orders one wave's LDS writes before its own later LDS reads (no other wave involved): the DS
// instructions of a wave execute in order, so a wavefront-scope fence (the compiler's ordering and
// the lgkm wait) stands in for a workgroup barrier when every element a wave reads next was written
// by that same wave.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Padded LDS blocks of the compile-time passes: 4 spare u64 after every 32, so that the
// set patterns of the chunk plans (element distance 1, 4 or 8 inside a run of 32, or a
// multiple of 32) fall on distinct banks for ds_read_b64 / ds_write_b64 (unpadded, the
// distance-4 sets were 8-way conflicts: 9.3 extra LDS cycles per instruction measured).
// A set's elements are j0 + m D with D = 2^dLog, j0 mod D < D and the group aligned to
// D M, so element m sits at lpad(j0) + lofs<D>(m): the run crossings depend on m only.
__device__ __forceinline__ uint32_t lpad(uint32_t i) { return i + ((i >> 5) << 2); }
template <int D>
__device__ constexpr uint32_t lofs(int m) {
  return (uint32_t)(m * D + (((m * D) >> 5) << 2));
}
constexpr uint32_t lpad_size(int BL) { return (1u << BL) + (1u << (BL - 3)); }

// ---- compile-time block passes over per-block twiddle tables ---------------
// For blocks of 2^BL elements (BL = ntt_block_log), block b owns the twiddle slice
// tb = tw_*_blk[t][b << BL]: local stage l (the l-th of the block's stages, in the
// transform's own order) and group i sit at tb[2^l + i] as one 16-byte {w, w'} pair
// (DeviceTables::tw_fwd_blk / tw_inv_blk).  Every shift below is a compile-time constant
// and every twiddle address is a block-uniform base plus a 32-bit offset: the generic
// passes above spend ~40 VALU instructions per butterfly, mostly on 64-bit index math.
//
// Forward chunk of KC stages starting at local half-size 2^H0: set s -> g = s >> dLog,
// j0 = g 2^(H0+1) + (s mod 2^dLog), elements j0 + m 2^dLog (dLog = H0 - KC + 1); its
// stage-i twiddles are tb[2^l + g 2^i + gs], gs < 2^i, l = BL - 1 - H0 + i.
//
// Reduction schedule: the stage at local half-size 2^h reduces its x inputs iff h is
// even, so the block's last stage (h = 0) always does: inputs below 12q (the columns
// pass leaves < 8q), outputs below 12q, never above 16q in between (ct_bfly_s).
// NORED (towers with q < 2^57, kNoRedQ): no reductions at all — a block's 11 stages add at
// most 44q to inputs below 17q (enc_cols_fused<..> leaves its NORED towers unreduced too), and
// 65q < 2^64 for the combine that follows.
template <int BL, int H0, int KC, bool NORED = false>
__device__ __forceinline__ void fwd_set_ct(uint64_t (&x)[1 << KC], uint32_t g,
                                           const ulonglong2* __restrict__ tb, uint64_t q,
                                           uint64_t n8q) {
#pragma unroll
  for (int i = 0; i < KC; ++i) {
    const int hm = 1 << (KC - 1 - i);
    const ulonglong2* __restrict__ tw = tb + (1u << (BL - 1 - H0 + i)) + (g << i);
#pragma unroll
    for (int gs = 0; gs < (1 << i); ++gs) {
      const ulonglong2 W = tw[gs];
#pragma unroll
      for (int mm = 0; mm < hm; ++mm) {
        if (!NORED && ((H0 - i) & 1) == 0)
          ct_bfly_s<true>(x[gs * 2 * hm + mm], x[gs * 2 * hm + mm + hm], W.x, W.y, q, n8q);
        else
          ct_bfly_s<false>(x[gs * 2 * hm + mm], x[gs * 2 * hm + mm + hm], W.x, W.y, q, n8q);
      }
    }
  }
}
// One forward chunk over all 2^(BL-KC) sets of the block (NS per thread): Load(j) gives
// element j, Store(r, j0, x) receives set r's transformed elements (positions j0 + m 2^dLog).
template <int BL, int H0, int KC, bool NORED = false, class Load, class Store>
__device__ __forceinline__ void fwd_chunk_ct(const ulonglong2* __restrict__ tb, uint64_t q,
                                             uint64_t n8q, Load ld, Store st) {
  constexpr int M = 1 << KC, dLog = H0 - KC + 1, NS = (1 << (BL - KC)) / 256;
  static_assert(NS >= 1 && dLog >= 0, "chunk plan");
#pragma unroll
  for (int r = 0; r < NS; ++r) {
    const uint32_t s = threadIdx.x + 256u * r;
    const uint32_t g = (H0 == BL - 1) ? 0u : s >> dLog;  // first chunk: one group
    const uint32_t j0 = (g << (H0 + 1)) + (s & ((1u << dLog) - 1));
    const uint32_t pj0 = lpad(j0);
    uint64_t x[M];
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = ld(j0 + (m << dLog), pj0 + lofs<(1 << dLog)>(m));
    fwd_set_ct<BL, H0, KC, NORED>(x, g, tb, q, n8q);
    st(r, j0, pj0, x);
  }
}
// One polynomial block's forward stages at compile-time shape (the chunk plan of
// ntt_fwd_blocks_enc_ct): the first chunk reads src (2^BL residues below 12q) straight into
// registers, two chunks go through the padded LDS block sm, and the last chunk hands each
// thread's 2^K4 contiguous outputs (below 12q; block offsets j0 ..) to fin(j0, x) from registers.
template <int BL, int K1, int K2, int K3, int K4, class Fin>
__device__ __forceinline__ void fwd_block_pass_ct(const uint64_t* __restrict__ src,
                                                  const ulonglong2* __restrict__ tb, uint64_t q, uint64_t n8q,
                                                  uint64_t* sm, Fin fin) {
  static_assert(K1 + K2 + K3 + K4 == BL, "chunk plan must cover the block");
  constexpr int M1 = 1 << K1, NS1 = (1 << (BL - K1)) / 256, D1 = BL - K1;
  constexpr int ML = 1 << K4, NSL = (1 << (BL - K4)) / 256;
  const auto lds_ld = [&](uint32_t, uint32_t pj) { return sm[pj]; };
#pragma unroll
  for (int r = 0; r < NS1; ++r) {
    uint64_t x[M1];
#pragma unroll
    for (int m = 0; m < M1; ++m) x[m] = src[threadIdx.x + 256u * r + (m << D1)];
    fwd_set_ct<BL, BL - 1, K1>(x, 0u, tb, q, n8q);
    const uint32_t p0 = lpad(threadIdx.x + 256u * r);
#pragma unroll
    for (int m = 0; m < M1; ++m) sm[p0 + lofs<(1 << D1)>(m)] = x[m];
  }
  __syncthreads();
  fwd_chunk_ct<BL, BL - 1 - K1, K2>(tb, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K2); ++m) sm[pj0 + lofs<(1 << (BL - K1 - K2))>(m)] = x[m];
  });
  __syncthreads();
  fwd_chunk_ct<BL, BL - 1 - K1 - K2, K3>(tb, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K3); ++m) sm[pj0 + lofs<(1 << (BL - K1 - K2 - K3))>(m)] = x[m];
  });
  __syncthreads();
#pragma unroll
  for (int r = 0; r < NSL; ++r) {
    const uint32_t g = threadIdx.x + 256u * r, j0 = g << K4, pj0 = lpad(j0);
    uint64_t x[ML];
#pragma unroll
    for (int m = 0; m < ML; ++m) x[m] = sm[pj0 + m];
    fwd_set_ct<BL, K4 - 1, K4>(x, g, tb, q, n8q);
    fin(j0, x);
  }
}

}  // namespace shelfi
