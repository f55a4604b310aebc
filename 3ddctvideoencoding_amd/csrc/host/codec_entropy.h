/* codec_entropy.h -- the codec's entropy stage (diagonal-slice order -> signed Exp-Golomb -> zlib),
 * stream-compatible with the reference C codec (encoder.c:60-86,241-274 / decoder.c:61-83,209-244):
 * one zlib stream (Z_BEST_COMPRESSION); per stack deflate(Z_NO_FLUSH) of the complete Exp-Golomb
 * bytes with the partial byte carried to the next stack; the last stack deflated with Z_FINISH
 * including its partial byte (+1).  Internal to libdct3dcodec (exported for the tests). */
#ifndef DCT3D_CODEC_ENTROPY_H_
#define DCT3D_CODEC_ENTROPY_H_

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dct3d_entropy_enc dct3d_entropy_enc;
typedef struct dct3d_entropy_dec dct3d_entropy_dec;

/* sink: FILE* (out) or, if out == NULL, an internal growable memory buffer */
dct3d_entropy_enc *dct3d_entropy_enc_create(int width, int height, int depth, FILE *out);
/* Optional, before the first push: deflate with `threads` worker threads (threads <= 1: the single zlib
 * stream, byte-identical to the reference encoder's .bin -- the default).  The parallel form cuts the
 * input into chunks of chunk_bytes (0: 256 KiB), deflates each at level 9 primed with the preceding
 * 32 KiB, joins them with sync flushes inside one zlib stream: a different .bin whose inflated payload
 * is the reference's. */
int dct3d_entropy_enc_set_threads(dct3d_entropy_enc *e, int threads, size_t chunk_bytes);
/* q: one stack of cubes, cube-major int32; is_last selects Z_FINISH (encoder.c:266-271) */
int dct3d_entropy_enc_push(dct3d_entropy_enc *e, const int32_t *q, int is_last);
/* the stream's current partial byte and the bits used in it (0..7): the carry for a stream built
 * elsewhere (the device Exp-Golomb stage, dct3d_encode_eg) */
void dct3d_entropy_enc_carry(const dct3d_entropy_enc *e, uint8_t *byte, int *bits);
/* appends an Exp-Golomb stream that starts with the carry above: total_bits bits (carry included) in
 * `bytes`; deflates its complete bytes (Z_NO_FLUSH) and keeps the partial byte, or, when is_last,
 * deflates them + the partial byte with Z_FINISH (encoder.c:263-274) */
int dct3d_entropy_enc_push_stream(dct3d_entropy_enc *e, const unsigned char *bytes, uint64_t total_bits, int is_last);
const unsigned char *dct3d_entropy_enc_memory(const dct3d_entropy_enc *e, size_t *len);
void dct3d_entropy_enc_destroy(dct3d_entropy_enc *e);

/* source: FILE* (in) or, if in == NULL, the memory block [mem, mem+len) */
dct3d_entropy_dec *dct3d_entropy_dec_create(int width, int height, int depth, FILE *in, const unsigned char *mem,
                                            size_t len);
/* fills one stack of cubes (cube-major int32); returns 0, or -1 on a truncated/corrupt stream */
int dct3d_entropy_dec_pull(dct3d_entropy_dec *d, int32_t *q);
/* the unconsumed inflated bytes (at least `need` unless the stream ends first) and the bit of the
 * first byte where the next code starts (0..7): the input of a device decode (dct3d_decode_eg) */
int dct3d_entropy_dec_window(dct3d_entropy_dec *d, size_t need, const unsigned char **p, size_t *len, int *bit);
/* consumes `bits` bits counted from the window's first byte (the window's start bit included) */
void dct3d_entropy_dec_consume(dct3d_entropy_dec *d, uint64_t bits);
/* 1 when the compressed input is exhausted (no more bytes will appear in the window) */
int dct3d_entropy_dec_eof(const dct3d_entropy_dec *d);
void dct3d_entropy_dec_destroy(dct3d_entropy_dec *d);

/* whole-buffer helpers (tests): q = n_stacks stacks cube-major */
int dct3d_codec_entropy_encode(const int32_t *q, int width, int height, int n_stacks, int depth,
                               unsigned char **out, size_t *out_len);
int dct3d_codec_entropy_decode(const unsigned char *bin, size_t len, int width, int height, int n_stacks, int depth,
                               int32_t *q);
int dct3d_codec_entropy_encode_mt(const int32_t *q, int width, int height, int n_stacks, int depth, int threads,
                                  size_t chunk_bytes, unsigned char **out, size_t *out_len);
void dct3d_codec_free(void *p);

#ifdef __cplusplus
}
#endif

#endif
