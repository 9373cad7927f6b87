/*
 * standard_attention.c -- C/OpenMP CPU oracle.  TEST INFRASTRUCTURE ONLY.
 *
 * Restates standard_attention_cpu (common/standard.h:28-102 of
 * tyler-utah/exploring_flash_attention): naive attention over [B,H,L,d], OpenMP over
 * (b,h) pairs (:41 collapse(2)), one L x L fp32 score buffer per head (:52), fp32
 * arithmetic over 16-bit storage (:14-22 DATA_TO_FLOAT / FLOAT_TO_DATA).  The reference
 * header includes cuda_runtime.h / cuda_fp16.h and cannot be compiled in this image, so
 * this restatement carries its own half / bfloat16 conversions (round-to-nearest-even).
 *
 * Also restates the CUDA drivers' input generator initialize_random
 * (flash_attention_v1/CUDA/driver.cu:71-75): srand(seed); x = rand()/RAND_MAX*2-1,
 * rounded to the storage type, so tests can rebuild the drivers' exact inputs.
 *
 * dtype codes match include/fa_mi355x.h: 0 = fp16, 1 = bf16, 2 = fp32.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static float h2f(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000) << 16, exp = (h >> 10) & 0x1f, man = h & 0x3ff, bits;
    if (exp == 0) {
        if (man == 0) {
            bits = sign;
        } else { /* subnormal: normalise */
            int e = -1;
            do { man <<= 1; ++e; } while (!(man & 0x400));
            bits = sign | ((uint32_t)(127 - 15 - e) << 23) | ((man & 0x3ff) << 13);
        }
    } else if (exp == 31) {
        bits = sign | 0x7f800000u | (man << 13);
    } else {
        bits = sign | ((exp + 127 - 15) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

static uint16_t f2h(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000;
    int32_t exp = (int32_t)((x >> 23) & 0xff) - 127 + 15;
    uint32_t man = x & 0x7fffff;
    if (((x >> 23) & 0xff) == 0xff) return (uint16_t)(sign | 0x7c00 | (man ? 0x200 : 0));
    if (exp >= 31) return (uint16_t)(sign | 0x7c00);
    if (exp <= 0) {
        if (exp < -10) return (uint16_t)sign;
        man |= 0x800000;
        uint32_t shift = (uint32_t)(14 - exp);
        uint32_t half = 1u << (shift - 1), rem = man & ((1u << shift) - 1);
        uint32_t r = man >> shift;
        if (rem > half || (rem == half && (r & 1))) ++r;
        return (uint16_t)(sign | r);
    }
    uint32_t r = (uint32_t)(exp << 10) | (man >> 13), rem = man & 0x1fff;
    if (rem > 0x1000 || (rem == 0x1000 && (r & 1))) ++r; /* may carry into exponent: ok */
    return (uint16_t)(sign | r);
}

static float b2f(uint16_t b) {
    uint32_t bits = (uint32_t)b << 16;
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

static uint16_t f2b(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    if ((x & 0x7fffffff) > 0x7f800000) return (uint16_t)((x >> 16) | 0x40);
    return (uint16_t)((x + 0x7fff + ((x >> 16) & 1)) >> 16);
}

static float load(const void* p, int64_t i, int dtype) {
    if (dtype == 0) return h2f(((const uint16_t*)p)[i]);
    if (dtype == 1) return b2f(((const uint16_t*)p)[i]);
    return ((const float*)p)[i];
}

static void store(void* p, int64_t i, float v, int dtype) {
    if (dtype == 0) ((uint16_t*)p)[i] = f2h(v);
    else if (dtype == 1) ((uint16_t*)p)[i] = f2b(v);
    else ((float*)p)[i] = v;
}

/* Round float values to the storage type (fp16 / bf16) and back, in place. */
void oracle_round_to(float* x, int64_t n, int dtype) {
    for (int64_t i = 0; i < n; ++i) {
        if (dtype == 0) x[i] = h2f(f2h(x[i]));
        else if (dtype == 1) x[i] = b2f(f2b(x[i]));
    }
}

/* Convert float <-> 16-bit storage. */
void oracle_to_storage(const float* x, void* out, int64_t n, int dtype) {
    for (int64_t i = 0; i < n; ++i) store(out, i, x[i], dtype);
}
void oracle_from_storage(const void* in, float* x, int64_t n, int dtype) {
    for (int64_t i = 0; i < n; ++i) x[i] = load(in, i, dtype);
}

/* initialize_random of the CUDA drivers: U[-1, 1] from glibc rand() after srand(seed). */
void oracle_driver_random(float* out, int64_t n, unsigned seed_or_neg1, int reseed) {
    if (reseed) srand(seed_or_neg1);
    for (int64_t i = 0; i < n; ++i) out[i] = ((float)rand() / RAND_MAX) * 2.0f - 1.0f;
}

/* standard_attention_cpu: q,k,v,o [B,H,L,d] in storage type dtype. */
void oracle_standard_attention(const void* Q, const void* K, const void* V, void* O, int B, int H,
                               int L, int d, int dtype) {
    const float scale = 1.0f / sqrtf((float)d);
#pragma omp parallel for collapse(2) schedule(dynamic)
    for (int b = 0; b < B; b++) {
        for (int h = 0; h < H; h++) {
            const int64_t base = ((int64_t)b * H + h) * (int64_t)L * d;
            float* s = (float*)malloc(sizeof(float) * (size_t)L * L);
            float* qrow = (float*)malloc(sizeof(float) * (size_t)d);
            float* kf = (float*)malloc(sizeof(float) * (size_t)L * d);
            float* vf = (float*)malloc(sizeof(float) * (size_t)L * d);
            for (int64_t i = 0; i < (int64_t)L * d; ++i) {
                kf[i] = load(K, base + i, dtype);
                vf[i] = load(V, base + i, dtype);
            }
            for (int i = 0; i < L; i++) {
                for (int c = 0; c < d; ++c) qrow[c] = load(Q, base + (int64_t)i * d + c, dtype);
                for (int j = 0; j < L; j++) {
                    float acc = 0.0f;
                    for (int c = 0; c < d; c++) acc += qrow[c] * kf[(int64_t)j * d + c];
                    s[(int64_t)i * L + j] = acc * scale;
                }
            }
            for (int i = 0; i < L; i++) {
                float* row = s + (int64_t)i * L;
                float mx = row[0];
                for (int j = 1; j < L; j++) mx = row[j] > mx ? row[j] : mx;
                float sum = 0.0f;
                for (int j = 0; j < L; j++) {
                    row[j] = expf(row[j] - mx);
                    sum += row[j];
                }
                for (int j = 0; j < L; j++) row[j] /= sum;
            }
            for (int i = 0; i < L; i++) {
                for (int c = 0; c < d; c++) {
                    float acc = 0.0f;
                    for (int j = 0; j < L; j++) acc += s[(int64_t)i * L + j] * vf[(int64_t)j * d + c];
                    store(O, base + (int64_t)i * d + c, acc, dtype);
                }
            }
            free(vf);
            free(kf);
            free(qrow);
            free(s);
        }
    }
}
