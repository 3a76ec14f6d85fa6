// host_arith_check.hip — TEST INFRASTRUCTURE (tests/test_host_arith.py).
//
// Compiles the product's field arithmetic (cudabulletproof_amd/csrc/fe25519_dev.h, whose
// functions are __host__ __device__; the host pass takes the C product, the device pass the
// gfx950 asm columns) as HOST code and compares it with the oracle (oracle/bp_oracle.c) on
// edge-heavy seeded inputs: fe_add, fe_sub, fe_mul (product + fold), fe_canon (tobytes),
// fe_sq (dedicated squaring vs mul(f, f)), fe_invert.  Prints "<op> <mismatches>" per op; exit status 1 on any mismatch.
#include <cstdio>
#include <cstring>

#include "../cudabulletproof_amd/csrc/fe25519_dev.h"
#include "../oracle/bp_oracle.h"

using bp::fe;

static uint64_t rng_state;
static uint64_t next64() {   // splitmix64
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Limb values that sit on the reference's lossy-carry edges.
static uint64_t edge_limb(int which) {
    static const uint64_t E[] = {0, 1, 2, 18, 19, 20, 0xFFFFFFFFFFFFFFEDull, 0xFFFFFFFFFFFFFFECull,
                                 0xFFFFFFFFFFFFFFEEull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFEull,
                                 0x7FFFFFFFFFFFFFFFull, 0x8000000000000000ull, 0x7FFFFFFFFFFFFFFEull,
                                 0xFFFFFFFF00000000ull, 0x00000000FFFFFFFFull,
                                 // x with lo64(19 x) = 2^64-1 (the fold's wrap case)
                                 0x79435E50D79435E5ull};
    return E[which % (sizeof(E) / sizeof(E[0]))];
}

static fe gen(int mode) {
    fe f;
    for (int i = 0; i < 4; i++) {
        uint64_t r = next64();
        switch (mode) {
            case 0: f.v[i] = next64(); break;
            case 1: f.v[i] = (r & 3) ? edge_limb((int)(r >> 8)) : next64(); break;
            default: f.v[i] = edge_limb((int)(r >> 8)); break;
        }
    }
    return f;
}

static bool same(const fe& a, const orc_fe& b) { return memcmp(a.v, b.v, 32) == 0; }

int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 200000;
    rng_state = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1;
    // sanity: the wrap-case constant really has 19x = -1 mod 2^64
    if ((uint64_t)(0x79435E50D79435E5ull * 19ull) != ~0ull) {
        printf("bad edge constant %llx\n", (unsigned long long)(0x79435E50D79435E5ull * 19ull));
    }
    long bad_sq = 0, bad_add = 0, bad_sub = 0, bad_mul = 0, bad_canon = 0, bad_inv = 0, bad_fold = 0;
    for (long it = 0; it < n; it++) {
        int mode = (int)(it % 3);
        fe f = gen(mode), g = gen((mode + 1) % 3);
        orc_fe of, og, r;
        memcpy(of.v, f.v, 32);
        memcpy(og.v, g.v, 32);
        orc_fe_add(&r, &of, &og);
        bad_add += !same(bp::fe_add(f, g), r);
        orc_fe_sub(&r, &of, &og);
        bad_sub += !same(bp::fe_sub(f, g), r);
        orc_fe_mul(&r, &of, &og);
        bad_mul += !same(bp::fe_mul(f, g), r);
        orc_fe_mul(&r, &of, &of);
        bad_sq += !same(bp::fe_sq(f), r);   // dedicated squaring == mul(f, f)
        uint8_t bytes[32];
        orc_fe_tobytes(bytes, &of);
        fe c = bp::fe_canon(f);
        bad_canon += memcmp(c.v, bytes, 32) != 0;   // little-endian limbs == tobytes bytes
        // fold directly on arbitrary 512-bit inputs (covers t_{i+4} = the wrap constant)
        uint64_t t[8];
        for (int i = 0; i < 8; i++) t[i] = (it & 1) ? edge_limb((int)(next64() >> 8)) : next64();
        fe ff = bp::fe_fold512(t);
        // oracle: fold == mul of (t_lo, 1) + ... is not expressible; emulate the reference fold
        {
            uint64_t h[4], cy;
            uint64_t cc = t[4] * 19ull;
            h[0] = t[0] + cc; cy = h[0] < cc;
            for (int i = 1; i < 4; i++) { cc = t[i + 4] * 19ull + cy; h[i] = t[i] + cc; cy = h[i] < cc; }
            orc_fe hh;
            memcpy(hh.v, h, 32);
            // condition: cy || h >= p, then the lossy "- p" == add(h, 0) with carry flag
            orc_fe zero = {{0, 0, 0, 0}}, viaadd;
            orc_fe_add(&viaadd, &hh, &zero);   // add(h, 0) applies exactly "if (h >= p) lossy - p"
            if (cy) {   // carry case: the lossy - p unconditionally (closed form of :62-66)
                uint64_t d[4], br1 = h[0] < 0xFFFFFFFFFFFFFFEDull;
                d[0] = h[0] + 19; d[1] = h[1] + 1 - br1;
                uint64_t br2 = (br1 == 0) & (h[1] != ~0ull);
                d[2] = h[2] + 1 - br2;
                uint64_t br3 = (br2 == 0) & (h[2] != ~0ull);
                d[3] = h[3] - 0x7FFFFFFFFFFFFFFFull - br3;
                memcpy(viaadd.v, d, 32);
            }
            bad_fold += !same(ff, viaadd);
        }
        if (it % 64 == 0) {
            orc_fe_invert(&r, &of);
            bad_inv += !same(bp::fe_invert(f), r);
        }
    }
    printf("add %ld\nsub %ld\nmul %ld\nsq %ld\ncanon %ld\nfold %ld\ninvert %ld\n", bad_add, bad_sub, bad_mul,
           bad_sq, bad_canon, bad_fold, bad_inv);
    return (bad_add | bad_sub | bad_mul | bad_sq | bad_canon | bad_fold | bad_inv) ? 1 : 0;
}
