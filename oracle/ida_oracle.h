/*
 * ida_oracle.h -- CPU restatement of the reference's Rabin IDA
 * (src/ida/ida.cpp, src/ida/matrix_math.cpp).  TEST INFRASTRUCTURE ONLY; see
 * chord_oracle.h and ida_oracle.c for the rules and the int32 wrap note.
 *
 * Layout of the batched forms (the same as the engine's cx_ida_*):
 *   block b = data[offsets[b] .. offsets[b+1]), S_b = ceil(len_b / m) segments,
 *   seg_offsets = prefix sums of S_b;
 *   encode: fragment i of block b = frags[n*seg_offsets[b] + i*S_b .. + S_b)
 *   decode: m fragment rows of block b at frags[m*seg_offsets[b] ..], their
 *           1-based indices at indices[b*m ..]; values out at out[m*seg_offsets[b]..],
 *           kept length out_len[b].
 */
#ifndef IDA_ORACLE_H
#define IDA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void or_ida_encoding_matrix(int n, int m, int p, int32_t *E);
int or_ida_vandermonde_inverse(const int *basis, int m, int p, int32_t *out);
void or_ida_encode(const uint8_t *data, size_t len, int n, int m, int p, uint16_t *frags);
long or_ida_decode(const uint16_t *frags, size_t S, const int *idx, int m, int p, uint16_t *out);
void or_ida_encode_batch(const uint8_t *data, const uint64_t *offsets, size_t blocks, int n, int m,
                         int p, uint16_t *frags);
int or_ida_decode_batch(const uint16_t *frags, const uint64_t *seg_offsets, const uint8_t *indices,
                        size_t blocks, int m, int p, uint16_t *out, uint64_t *out_len);

#ifdef __cplusplus
}
#endif
#endif /* IDA_ORACLE_H */
