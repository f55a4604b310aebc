/* dct3d_diag.h -- libdct3d_diag.so: measurement and test support for libdct3d.so, NOT the product
 * path.  Nothing in libdct3d.so or the codec calls these; bench.py and the tests do.  Every call
 * runs on the stream of the given ctx (dct3d_ctx_info), after the ctx's earlier work. */
#ifndef DCT3D_DIAG_H
#define DCT3D_DIAG_H

#include "dct3d.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------------------
 * Benchmark / test support: integer-only deterministic synthetic frames, identical to the
 * Python generator (3ddctvideoencoding_amd.synthetic).  For global pixel index
 * idx = ((frame0 + f) * height + y) * width + x:
 *   kind 0 ("ramp"):    clamp(128 + ((3x + 5y + 7(frame0+f)) & 63) - 32 + (splitmix64(seed ^ idx) & 15))
 *   kind 1 ("uniform"): splitmix64(seed ^ idx) & 255
 * ------------------------------------------------------------------------------------------- */
int dct3d_fill_synthetic_dev(dct3d_ctx *ctx, uint8_t *d_frames, int width, int height, int n_frames,
                             uint64_t seed, int64_t frame0, int kind);

/* Bandwidth calibration (bench support): the encode's traffic pattern without the transform, on the
 * context stream.  mode 0: d_in u8 [n_px] -> d_out int32 [n_px] (1 B read : 4 B written, NT stores);
 * mode 1: copy n_px bytes; mode 2: write 4*n_px bytes; mode 3: read n_px bytes; modes 4/5: copy /
 * write with plain (temporal) stores.  n_px % 16 == 0. */
int dct3d_bandwidth_probe_dev(dct3d_ctx *ctx, const uint8_t *d_in, void *d_out, size_t n_px, int mode);

/* Memory-only twin of dct3d_encode_stacks_dev (bench support; d_q receives NOT a DCT): the encode
 * kernel's row loads, LDS staging and 1 KiB non-temporal stores of the same cubes, without the
 * transform, quantisation or certification.  Its rate is the ceiling the encode's own traffic
 * reaches on this device. */
int dct3d_encode_memonly_dev(dct3d_ctx *ctx, const uint8_t *d_raster, int width, int height, int n_stacks,
                             int32_t *d_q);
/* The encode kernel split in two (bench support; d_q receives NOT a DCT): mode 1 = memory only (as
 * dct3d_encode_memonly_dev), mode 2 = compute only (8x8x8 contexts: rows made from the lane and cube
 * indices instead of the loads, the whole transform / quantise / certify / staging, no stores). */
int dct3d_encode_diag_dev(dct3d_ctx *ctx, const uint8_t *d_raster, int width, int height, int n_stacks,
                          int32_t *d_q, int mode);
/* As dct3d_encode_diag_dev; mode 3 (8x8x8) = the product encode (d_q IS the encode) with a timeline:
 * d_trace[4 w .. 4 w + 3] of wave w = {start, transform done, stores issued} on the 100 MHz
 * s_memrealtime clock and (XCC_ID << 32 | HW_ID).  d_trace: 32 bytes per 4 cubes. */
int dct3d_encode_trace_dev(dct3d_ctx *ctx, const uint8_t *d_raster, int width, int height, int n_stacks,
                           int32_t *d_q, int mode, uint64_t *d_trace);

/* Traversal sweep (the 4K shard's read pattern): the 8x8x8 encode with its waves walking the
 * cubes in vertical strips of strip_w cubes (strip-major: stack, strip, block row, column in the strip)
 * instead of the product's row-major order; the output is the same cube-major array.  mode 1 = memory
 * only (as dct3d_encode_diag_dev mode 1; d_q is NOT a DCT), mode 0 = the full encode (d_q IS the encode,
 * rare paths included, no replay counters).  strip_w: a multiple of 4 dividing width / 8. */
int dct3d_encode_strip_dev(dct3d_ctx *ctx, const uint8_t *d_raster, int width, int height, int n_stacks,
                           int32_t *d_q, int mode, int strip_w);

/* The decode kernel split in two (bench support; d_raster receives NOT a decode): mode 1 = memory only
 * (the same staged loads and raster stores, no transform), mode 2 = compute only (no global loads, no
 * stores).  The decode's time read against both shows how far its memory and its fp64 issue overlap
 * (DESIGN.md §4).  8x8x8 and 8x8x4 contexts. */
int dct3d_decode_diag_dev(dct3d_ctx *ctx, const int32_t *d_q, int width, int height, int n_stacks,
                          uint8_t *d_raster, int mode);

#ifdef __cplusplus
}
#endif

#endif /* DCT3D_DIAG_H */
