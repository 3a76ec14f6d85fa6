// sha256_dev.h — FIPS 180-4 SHA-256 on the device, for the Fiat-Shamir challenges of the
// verify path (bulletproof_challenge.cu:6-77, cuda_range_proof_verify.cu:185-205) and the
// hash term of the tolerant accept rule (cuda_range_proof_verify.cu:330-344).
// One lane hashes one message; messages on this path are < 256 bytes.
#pragma once
#include "fe25519_dev.h"
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bp {

__device__ __constant__ static const uint32_t kSHA[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t sha_ror(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

__device__ __forceinline__ void sha_compress(uint32_t st[8], const uint32_t in[16]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = in[i];
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            uint32_t s0 = sha_ror(w15, 7) ^ sha_ror(w15, 18) ^ (w15 >> 3);
            uint32_t s1 = sha_ror(w2, 17) ^ sha_ror(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        uint32_t t1 = h + (sha_ror(e, 6) ^ sha_ror(e, 11) ^ sha_ror(e, 25)) + ((e & f) ^ (~e & g)) + kSHA[i] + wi;
        uint32_t t2 = (sha_ror(a, 2) ^ sha_ror(a, 13) ^ sha_ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// ------------------------------------------------------------------ register-resident messages
// Every message on this path has a fixed layout (tags, 32-byte field elements), so each byte's
// position is a compile-time constant: `shaw` places 4-byte groups at template byte offsets, and
// all block indexing is constant, so the state and the block stay in VGPRs.  (Round 6: the earlier
// byte-at-a-time context appended at a run-time position, which put its block in scratch memory
// and made every byte a dependent scratch read-modify-write on the challenge chains of the
// latency-bound ticks.)
struct shaw {
    uint32_t st[8];
    uint32_t b[16];   // the current block; word k is assigned before any byte of it is OR-ed in
};

__device__ __forceinline__ void shaw_init(shaw& c) {
    c.st[0] = 0x6a09e667; c.st[1] = 0xbb67ae85; c.st[2] = 0x3c6ef372; c.st[3] = 0xa54ff53a;
    c.st[4] = 0x510e527f; c.st[5] = 0x9b05688c; c.st[6] = 0x1f83d9ab; c.st[7] = 0x5be0cd19;
}

// NB (1..4) message bytes at byte offset P, as the top NB bytes of w (big-endian, low bytes zero)
template <int P, int NB = 4>
__device__ __forceinline__ void shaw_put(shaw& c, uint32_t w) {
    constexpr int off = P & 3, wi = (P >> 2) & 15;
    if constexpr (off == 0) c.b[wi] = w;
    else c.b[wi] |= w >> (8 * off);
    if constexpr ((P & 63) + NB >= 64) sha_compress(c.st, c.b);   // this put completes the block
    if constexpr (off + NB > 4) c.b[(wi + 1) & 15] = w << (32 - 8 * off);
}

template <int P, int I, int LEN>
__device__ __forceinline__ void shaw_str_at(shaw& c, const char* s) {
    if constexpr (I < LEN) {
        constexpr int nb = LEN - I < 4 ? LEN - I : 4;
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < nb; k++) w |= (uint32_t)(uint8_t)s[I + k] << (24 - 8 * k);
        shaw_put<P + I, nb>(c, w);
        shaw_str_at<P, I + 4, LEN>(c, s);
    }
}
// a string literal's characters (no terminator) at byte offset P
template <int P, int N>
__device__ __forceinline__ void shaw_str(shaw& c, const char (&s)[N]) {
    shaw_str_at<P, 0, N - 1>(c, s);
}

// 4 little-endian u64 limbs (fe25519_tobytes byte order) at byte offset P
template <int P>
__device__ __forceinline__ void shaw_limbs(shaw& c, const fe& f) {
    shaw_put<P + 0>(c, __builtin_bswap32((uint32_t)f.v[0]));
    shaw_put<P + 4>(c, __builtin_bswap32((uint32_t)(f.v[0] >> 32)));
    shaw_put<P + 8>(c, __builtin_bswap32((uint32_t)f.v[1]));
    shaw_put<P + 12>(c, __builtin_bswap32((uint32_t)(f.v[1] >> 32)));
    shaw_put<P + 16>(c, __builtin_bswap32((uint32_t)f.v[2]));
    shaw_put<P + 20>(c, __builtin_bswap32((uint32_t)(f.v[2] >> 32)));
    shaw_put<P + 24>(c, __builtin_bswap32((uint32_t)f.v[3]));
    shaw_put<P + 28>(c, __builtin_bswap32((uint32_t)(f.v[3] >> 32)));
}
template <int P>
__device__ __forceinline__ void shaw_fe_canon(shaw& c, const fe& f) {   // host fe25519_tobytes
    shaw_limbs<P>(c, fe_canon(f));
}

// Padding and length for an L-byte message; the digest as 4 little-endian u64 limbs.
template <int L>
__device__ __forceinline__ void shaw_final_limbs(shaw& c, uint64_t out[4]) {
    shaw_put<L, 1>(c, 0x80000000u);
    constexpr int q = (L + 1) & 63;        // bytes of the current block in use (0: the put compressed it)
    constexpr int w0 = q ? (q + 3) / 4 : 0;   // its first unassigned word
    if constexpr (q > 56) {                // no room for the length: zero the rest, a block of its own
#pragma unroll
        for (int k = w0; k < 16; k++) c.b[k] = 0;
        sha_compress(c.st, c.b);
#pragma unroll
        for (int k = 0; k < 14; k++) c.b[k] = 0;
    } else {
#pragma unroll
        for (int k = w0; k < 14; k++) c.b[k] = 0;
    }
    c.b[14] = 0;
    c.b[15] = (uint32_t)L * 8u;
    sha_compress(c.st, c.b);
#pragma unroll
    for (int i = 0; i < 4; i++)
        out[i] = (uint64_t)__builtin_bswap32(c.st[2 * i]) | ((uint64_t)__builtin_bswap32(c.st[2 * i + 1]) << 32);
}
template <int L>
__device__ __forceinline__ fe shaw_challenge(shaw& c) {   // generate_challenge: output[31] &= 0x7F
    fe r;
    shaw_final_limbs<L>(c, r.v);
    r.v[3] &= 0x7FFFFFFFFFFFFFFFull;
    return r;
}

// The path's messages (bulletproof_challenge.cu:24-77, cuda_range_proof_verify.cu:185-205, :330-344,
// bulletproof_range_proof.cu:560-566, :1636-1650)
// y = H("BulletproofYChal" || V.X V.Y A.X A.Y S.X S.Y || "y_ch")   (challenge.cu:24-44)
__device__ __forceinline__ fe chal_y(const ge& V, const ge& A, const ge& S) {
    shaw c;
    shaw_init(c);
    shaw_str<0>(c, "BulletproofYChal");
    shaw_fe_canon<16>(c, V.X); shaw_fe_canon<48>(c, V.Y);
    shaw_fe_canon<80>(c, A.X); shaw_fe_canon<112>(c, A.Y);
    shaw_fe_canon<144>(c, S.X); shaw_fe_canon<176>(c, S.Y);
    shaw_str<208>(c, "y_ch");
    return shaw_challenge<212>(c);
}
// z = H("BulletproofZChal" || y (raw limbs) || "z_ch")   (challenge.cu:47-58)
__device__ __forceinline__ fe chal_z(const fe& y) {
    shaw c;
    shaw_init(c);
    shaw_str<0>(c, "BulletproofZChal");
    shaw_limbs<16>(c, y);
    shaw_str<48>(c, "z_ch");
    return shaw_challenge<52>(c);
}
// x = H("BulletproofXChal" || T1.X T1.Y T2.X T2.Y || "xcha")   (challenge.cu:61-77: 4 bytes of "xchal")
__device__ __forceinline__ fe chal_x(const ge& T1, const ge& T2) {
    shaw c;
    shaw_init(c);
    shaw_str<0>(c, "BulletproofXChal");
    shaw_fe_canon<16>(c, T1.X); shaw_fe_canon<48>(c, T1.Y);
    shaw_fe_canon<80>(c, T2.X); shaw_fe_canon<112>(c, T2.Y);
    shaw_str<144>(c, "xcha");
    return shaw_challenge<148>(c);
}
// u_r = H("InnerProductChal" || transcript (raw limbs) || L.X || R.X)   (crv:185-205, rp.cu inner_product_prove)
__device__ __forceinline__ fe chal_ip(const fe& tr, const fe& Lx, const fe& Rx) {
    shaw c;
    shaw_init(c);
    shaw_str<0>(c, "InnerProductChal");
    shaw_limbs<16>(c, tr);
    shaw_fe_canon<48>(c, Lx);
    shaw_fe_canon<80>(c, Rx);
    return shaw_challenge<112>(c);
}
// the prover's IPA transcript start H("BulletproofIP" || t || taux || mu)   (rp.cu:1636-1650)
__device__ __forceinline__ fe chal_ip_start(const fe& t, const fe& taux, const fe& mu) {
    shaw c;
    shaw_init(c);
    shaw_str<0>(c, "BulletproofIP");
    shaw_fe_canon<13>(c, t);
    shaw_fe_canon<45>(c, taux);
    shaw_fe_canon<77>(c, mu);
    return shaw_challenge<109>(c);
}
// SHA-256 of four 32-byte values in raw limb order (the accept rule's hash term, crv:330-344; the
// method-3 challenge, rp.cu:560-566): the full digest, unmasked
__device__ __forceinline__ fe sha_4fe(const fe& a, const fe& b, const fe& d, const fe& e) {
    shaw c;
    shaw_init(c);
    shaw_limbs<0>(c, a); shaw_limbs<32>(c, b); shaw_limbs<64>(c, d); shaw_limbs<96>(c, e);
    fe r;
    shaw_final_limbs<128>(c, r.v);
    return r;
}

}  // namespace bp
