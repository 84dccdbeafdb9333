/*
 * ida_oracle.c -- CPU restatement of the reference's Rabin IDA (DHash payload
 * coding): src/ida/ida.cpp, src/ida/matrix_math.cpp, src/ida/data_block.cpp.
 *
 * TEST INFRASTRUCTURE ONLY (see chord_oracle.h): the parity checker for the
 * engine's cx_ida_* kernels; the product path never calls it.
 *
 * The reference computes in C++ `int` (Vector = std::vector<int>,
 * matrix_math.h:10).  Two places can leave int range:
 *   - ElementarySymmetricTransform (matrix_math.cpp:103-116) sums products of
 *     fragment indices without reduction: for (n, m) = (14, 10) a symmetric sum
 *     e_j (j < m) exceeds 2^31 for 7 of the 1001 fragment sets (those missing
 *     most of fragments 1-4);
 *   - the numerator step `row.back() * elt mod p + sign * el[j]`
 *     (matrix_math.cpp:139) adds to such a value.
 * We restate these as the compiled code runs them on x86-64: two's-complement
 * wrap-around (int32 arithmetic done in uint32).  No reference test decodes
 * from such a fragment set, so that corner is "parity unpinned"; every other
 * value stays in int range for p <= 46340 (the engine's limit).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ida_oracle.h"

/* int32 arithmetic with wrap-around (the compiled behaviour of `int`). */
static inline int32_t w_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t w_mul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

/* Modulo (matrix_math.cpp:21-24): (lhs % rhs + rhs) % rhs, C++ truncating %. */
static inline int32_t modp(int32_t lhs, int32_t rhs) { return (lhs % rhs + rhs) % rhs; }

/* ConstructEncodingMatrix (matrix_math.cpp:88-101): row a-1 = a^0..a^(m-1) mod p. */
void or_ida_encoding_matrix(int n, int m, int p, int32_t *E) {
    for (int a = 1; a <= n; ++a) {
        int32_t elt = 1;
        for (int i = 0; i < m; ++i) {
            E[(a - 1) * m + i] = elt;
            elt = modp(elt * a, p);
        }
    }
}

/* ModInverse (matrix_math.cpp:66-86): extended Euclid; -1 when not invertible. */
static int32_t mod_inverse(int32_t nn, int32_t p) {
    int32_t t = 0, new_t = 1, r = p, new_r = nn;
    while (new_r) {
        const int32_t q = r / new_r;
        int32_t tmp = t;
        t = new_t;
        new_t = tmp - q * new_t;
        tmp = r;
        r = new_r;
        new_r = tmp - q * new_r;
    }
    if (r > 1) return -1;
    if (t < 0) t += p;
    return t;
}

/* VandermondeInverse (matrix_math.cpp:103-168) for basis b[0..m): out is the
 * m x m matrix (row-major) the reference returns (the transpose of its
 * row-per-basis result).  Returns 0, or -1 when a denominator is not
 * invertible (the reference throws "N is not invertible"). */
int or_ida_vandermonde_inverse(const int *basis, int m, int p, int32_t *out) {
    /* ElementarySymmetricTransform(v = basis, m) */
    int32_t *el = (int32_t *)calloc((size_t)(m + 1) * (m + 1), sizeof(int32_t));
    int32_t *res = (int32_t *)malloc((size_t)m * m * sizeof(int32_t));
    if (!el || !res) {
        free(el);
        free(res);
        return -1;
    }
#define EL(i, j) el[(size_t)(i) * (m + 1) + (j)]
    for (int i = 1; i <= m; ++i) EL(1, i) = w_add(EL(1, i - 1), basis[i - 1]);
    for (int i = 2; i <= m; ++i)
        for (int j = i; j <= m; ++j) EL(i, j) = w_add(w_mul(EL(i - 1, j - 1), basis[j - 1]), EL(i, j - 1));
    /* result[i] = el[i].back(), i = 0..m (el[0] is all zeros) */
    int rc = 0;
    for (int i = 0; i < m && rc == 0; ++i) {
        int32_t prod = 1;
        const int32_t elt = basis[i];
        for (int j = 0; j < m; ++j)
            if (j != i) prod = modp(prod * (elt - basis[j]), p);
        const int32_t inv = mod_inverse(prod, p);
        if (inv < 0) {
            rc = -1;
            break;
        }
        /* numerators: row = {1}; cell = Modulo(Modulo(row.back()*elt, p) + sign*el[j], p) */
        int32_t row[64];
        row[0] = 1;
        int32_t sign = -1;
        for (int j = 1; j < m; ++j) {
            const int32_t a = modp(row[j - 1] * elt, p);
            row[j] = modp(w_add(a, w_mul(sign, EL(j, m))), p);
            sign = -sign;
        }
        /* reverse, scale by the inverse denominator */
        for (int j = 0; j < m; ++j) res[(size_t)i * m + j] = modp(row[m - 1 - j] * inv, p);
    }
#undef EL
    if (rc == 0)
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < m; ++j) out[(size_t)i * m + j] = res[(size_t)j * m + i];  /* Transpose */
    free(el);
    free(res);
    return rc;
}

/* IDA::Encode (ida.cpp:59-73) of one datum: segments of m values
 * (SplitToSegments, ida.cpp:177-190, zero-padded), fragment i value s =
 * InnerProduct(E[i], segment s) mod p (matrix_math.cpp:26-33).  frags is
 * n rows x S = ceil(len / m) values. */
void or_ida_encode(const uint8_t *data, size_t len, int n, int m, int p, uint16_t *frags) {
    int32_t E[64 * 64];
    or_ida_encoding_matrix(n, m, p, E);
    const size_t S = (len + (size_t)m - 1) / (size_t)m;
    for (size_t s = 0; s < S; ++s) {
        int32_t seg[64];
        for (int k = 0; k < m; ++k) {
            const size_t at = s * (size_t)m + (size_t)k;
            seg[k] = at < len ? (int32_t)data[at] : 0;
        }
        for (int i = 0; i < n; ++i) {
            int32_t sum = 0;
            for (int k = 0; k < m; ++k) sum += E[i * m + k] * seg[k];
            frags[(size_t)i * S + s] = (uint16_t)modp(sum, p);
        }
    }
}

/* IDA::Decode (ida.cpp:120-162) from m fragments (rows of S values) with
 * 1-based fragment indices idx[0..m): inverse Vandermonde of the indices times
 * the fragment matrix (MatrixProduct, matrix_math.cpp:35-55, reducing every
 * step), read column-wise, then trailing all-zero segments and the trailing
 * zeros of the last segment are dropped.  out receives up to m*S values;
 * returns the kept length, or -1 if the indices are not invertible.  (When
 * every value is zero the reference reads back() of an empty vector; we
 * return 0.) */
long or_ida_decode(const uint16_t *frags, size_t S, const int *idx, int m, int p, uint16_t *out) {
    int32_t inv[64 * 64];
    if (or_ida_vandermonde_inverse(idx, m, p, inv) != 0) return -1;
    long last = -1;
    for (size_t s = 0; s < S; ++s)
        for (int j = 0; j < m; ++j) {
            int32_t cell = 0;
            for (int k = 0; k < m; ++k)
                cell = modp(w_add(cell, w_mul(inv[j * m + k], (int32_t)frags[(size_t)k * S + s])), p);
            const size_t at = s * (size_t)m + (size_t)j;
            out[at] = (uint16_t)cell;
            if (cell != 0) last = (long)at;
        }
    return last + 1;
}

/* Batched forms over ragged blocks (the layout cx_ida_* use). */
void or_ida_encode_batch(const uint8_t *data, const uint64_t *offsets, size_t blocks, int n, int m,
                         int p, uint16_t *frags) {
    size_t seg = 0;
    for (size_t b = 0; b < blocks; ++b) {
        const size_t len = offsets[b + 1] - offsets[b];
        const size_t S = (len + (size_t)m - 1) / (size_t)m;
        or_ida_encode(data + offsets[b], len, n, m, p, frags + (size_t)n * seg);
        seg += S;
    }
}

int or_ida_decode_batch(const uint16_t *frags, const uint64_t *seg_offsets, const uint8_t *indices,
                        size_t blocks, int m, int p, uint16_t *out, uint64_t *out_len) {
    int idx[64];
    for (size_t b = 0; b < blocks; ++b) {
        const size_t S = seg_offsets[b + 1] - seg_offsets[b];
        for (int k = 0; k < m; ++k) idx[k] = indices[b * (size_t)m + k];
        const long L = or_ida_decode(frags + (size_t)m * seg_offsets[b], S, idx, m, p,
                                     out + (size_t)m * seg_offsets[b]);
        if (L < 0) return -1;
        out_len[b] = (uint64_t)L;
    }
    return 0;
}
