/* det_rand.c — TEST INFRASTRUCTURE ONLY.  Deterministic RAND_bytes for the drop-in demo
 * binary (oracle/_ref/complete_bulletproof_test_hip): block k = SHA256(seed_le64 || k_le64),
 * seed from $BP_RAND_SEED (default 1); the same stream as ref_harness.cc, so the demo's
 * 16-bit proof is the one in tests/golden/proofs_n16.npz (index 0). */
#include <stdint.h>
#include <stdlib.h>
#include <openssl/sha.h>

static uint64_t g_seed = 0, g_ctr = 0;
static unsigned char g_block[32];
static int g_avail = 0, g_init = 0;

int RAND_bytes(unsigned char* buf, int num) {
    if (!g_init) {
        const char* e = getenv("BP_RAND_SEED");
        g_seed = e ? strtoull(e, 0, 10) : 1;
        g_init = 1;
    }
    for (int i = 0; i < num; i++) {
        if (g_avail == 0) {
            unsigned char in[16];
            for (int k = 0; k < 8; k++) { in[k] = (unsigned char)(g_seed >> (8 * k)); in[8 + k] = (unsigned char)(g_ctr >> (8 * k)); }
            SHA256(in, 16, g_block);
            g_ctr++;
            g_avail = 32;
        }
        buf[i] = g_block[32 - g_avail];
        g_avail--;
    }
    return 1;
}
