/* CPU restatement of the sampler's counter-based RNG — TEST ORACLE ONLY.
 *
 * Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
 * SC'11), the generator torch's device RNG also uses.  The reference draws
 * with torch.multinomial (transformers `_sample`), whose stream cannot be
 * reproduced by a device Gumbel-max sampler; the product's sampler therefore
 * defines its own documented stream (DESIGN.md §Sampler RNG) and this file is
 * the independent CPU statement of that stream:
 *
 *   key  = { seed_lo, seed_hi }
 *   ctr  = { j >> 2, row, offset_lo, offset_hi }
 *   word = philox(ctr, key)[j & 3]
 *   u    = ((word >> 8) + 0.5) * 2^-24          in (0, 1), exact in fp32
 *
 * Pinned by the published Philox4x32-10 known-answer vectors
 * (tests/golden/philox_kat.json).  Built by oracle/Makefile into
 * oracle/_build/libswh_oracle.so.
 */
#include <stdint.h>

static inline void mulhilo(uint32_t a, uint32_t b, uint32_t *hi, uint32_t *lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    *lo = (uint32_t)p;
}

void swh_ref_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(0xD2511F53u, c0, &hi0, &lo0);
        mulhilo(0xCD9E8D57u, c2, &hi1, &lo1);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Uniforms u[j], j in [0, V), of one sampler row: word (row & 3) of the
 * block at counter {j, row >> 2, offset} (swh_trl_amd/csrc/sampler.hip gumbel_at). */
void swh_ref_row_uniforms(uint64_t seed, uint64_t offset, int64_t row, int64_t V, float *u) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t j = 0; j < V; ++j) {
        uint32_t ctr[4] = {(uint32_t)j, (uint32_t)(row >> 2), (uint32_t)offset, (uint32_t)(offset >> 32)};
        uint32_t w[4];
        swh_ref_philox4x32_10(ctr, key, w);
        u[j] = ((float)(w[row & 3] >> 8) + 0.5f) * (1.0f / 16777216.0f);
    }
}
