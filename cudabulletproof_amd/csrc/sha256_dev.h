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

struct sha256_ctx {
    uint32_t st[8];
    uint32_t blk[16];   // current block, big-endian words
    uint32_t used;      // bytes in blk
    uint32_t total;     // message bytes so far
};

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

__device__ __forceinline__ void sha_init(sha256_ctx& c) {
    c.st[0] = 0x6a09e667; c.st[1] = 0xbb67ae85; c.st[2] = 0x3c6ef372; c.st[3] = 0xa54ff53a;
    c.st[4] = 0x510e527f; c.st[5] = 0x9b05688c; c.st[6] = 0x1f83d9ab; c.st[7] = 0x5be0cd19;
#pragma unroll
    for (int i = 0; i < 16; i++) c.blk[i] = 0;
    c.used = 0;
    c.total = 0;
}

__device__ __forceinline__ void sha_byte(sha256_ctx& c, uint32_t byte) {
    uint32_t wi = c.used >> 2, sh = 24 - 8 * (c.used & 3);
    c.blk[wi] |= (byte & 0xff) << sh;
    c.used++;
    c.total++;
    if (c.used == 64) {
        sha_compress(c.st, c.blk);
#pragma unroll
        for (int i = 0; i < 16; i++) c.blk[i] = 0;
        c.used = 0;
    }
}

__device__ __forceinline__ void sha_bytes(sha256_ctx& c, const uint8_t* p, int n) {
    for (int i = 0; i < n; i++) sha_byte(c, p[i]);
}

// 64-bit little-endian limb stream (fe25519_tobytes byte order)
__device__ __forceinline__ void sha_limbs(sha256_ctx& c, const uint64_t* v, int nlimbs) {
    for (int l = 0; l < nlimbs; l++)
        for (int k = 0; k < 8; k++) sha_byte(c, (uint32_t)(v[l] >> (8 * k)));
}

__device__ __forceinline__ void sha_str(sha256_ctx& c, const char* s) {
    for (; *s; s++) sha_byte(c, (uint8_t)*s);
}

// Finalize; the digest is returned as 4 little-endian u64 limbs (bytes 0..31 of the digest
// in fe25519_frombytes order).
__device__ __forceinline__ void sha_final_limbs(sha256_ctx& c, uint64_t out[4]) {
    uint32_t bits = c.total * 8;
    sha_byte(c, 0x80);
    c.total--;   // padding is not message
    while (c.used != 56) { sha_byte(c, 0); c.total--; }
    c.blk[14] = 0;
    c.blk[15] = bits;
    sha_compress(c.st, c.blk);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t w0 = c.st[2 * i], w1 = c.st[2 * i + 1];
        // digest bytes are big-endian words; limb = bytes[8i..8i+7] little-endian
        uint64_t lo = __builtin_bswap32(w0), hi = __builtin_bswap32(w1);
        out[i] = lo | (hi << 32);
    }
}

// host fe25519_tobytes (canonicalising) into the hash (challenge inputs, bulletproof_challenge.cu)
__device__ __forceinline__ void sha_fe_canon(sha256_ctx& c, const fe& f) {
    fe t = fe_canon(f);
    sha_limbs(c, t.v, 4);
}

// generate_challenge's digest as a field element: output[31] &= 0x7F (bulletproof_challenge.cu:20)
__device__ __forceinline__ fe challenge_digest(sha256_ctx& c) {
    fe r;
    sha_final_limbs(c, r.v);
    r.v[3] &= 0x7FFFFFFFFFFFFFFFull;
    return r;
}

}  // namespace bp
