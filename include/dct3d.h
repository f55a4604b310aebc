/*
 * dct3d.h -- C-ABI of the MI355X 3D-DCT hot path (libdct3d.so).
 *
 * Drop-in boundary for julianopiccoli/3dDCTVideoEncoding's per-stack device block.  The reference
 * C codec (3d-DCT-video-encoding-OpenCL/) does, per 8-frame stack:
 *     readCubes -> clEnqueueWriteBuffer -> dct_calculate_partial_sums -> dct_aggregate_partial_sums
 *     -> clEnqueueReadBuffer -> applyQuantization                       (encoder.c:206-260)
 *     applyDequantization -> clEnqueueWriteBuffer -> idct_calculate_partial_sums
 *     -> idct_aggregate_partial_sums -> clEnqueueReadBuffer -> writeCubes (decoder.c:246-295)
 * after a per-call OpenCL setup (encoder.c:147-197, decoder.c:153-202, OpenCLUtils.c:49-165).
 * Each entry point below names the reference region it replaces.
 *
 * Conventions (all entry points):
 *   - plain pointers and sizes, no framework types; 0 = DCT3D_OK, non-zero = DCT3D_E* code
 *     (the reference printf()s and returns 1, or exit(1)s inside OpenCLUtils.c; this library never
 *     prints and never exits -- the codec layer above prints, see codec.h);
 *   - a context owns its device buffers and its HIP stream (the reference creates its OpenCL objects
 *     per call and never releases them, encoder.c:165-197); one context per device, one host
 *     thread per context (a context is not thread-safe);
 *   - host-pointer entry points are synchronous on return (the reference's blocking
 *     clEnqueueWrite/ReadBuffer, encoder.c:209,254); *_dev entry points take device pointers and
 *     are asynchronous on the context stream (use dct3d_synchronize).  The context's own stream is a
 *     blocking stream (ordered with the legacy default stream); dct3d_ctx_set_stream selects another;
 *   - frame width must be a multiple of the block width and height of the block height
 *     (1080 = 135 * 8); the reference silently overruns otherwise, this library returns
 *     DCT3D_EINVAL.
 *
 * Layouts:
 *   raster  : u8 frames, frame-major, row-major (the raw grayscale file format, encoder.c:21-27);
 *             a "stack" is DCT_BLOCK_DEPTH consecutive frames.
 *   cubes   : cube-major: for each stack, block-row by, block-col bx, then (z, y, x) inside the cube
 *             (readCubes order, encoder.c:29-41; Java Encoder.java:75-89).
 *
 * Numerics (parity target = the reference Java codec, BASELINE.json north_star):
 *   - dct3d_encode_stacks*: quantised int32 coefficients equal to the Java path
 *       Math.round(DCT.apply(...)[k] / max(1, 5(x+y+z)))          (Encoder.java:82, DCT.java:41-59)
 *     bit for bit: computed in fp32 under a rigorous per-coefficient error bound; any coefficient
 *     whose quotient is within that bound of a rounding tie is recomputed by replaying the Java
 *     fold exactly (fp64, HashMap group order), and the DC from the exact integer cube sum.
 *   - dct3d_decode_stacks*: u8 pixels equal to the Java path (byte) clamp(InverseDCT(...))
 *     (InverseDCT.java:33-82, Decoder.java:112) bit for bit, same certify-or-replay scheme (fp64).
 *   - float outputs (dct_opt, dct3d_forward_f32, dct3d_inverse_f32): fp64 internal arithmetic;
 *     |err| <= 1e-9 * max(1, |value|) before the final rounding to the output type.
 */
#ifndef DCT3D_H_
#define DCT3D_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCT3D_OK 0
#define DCT3D_EINVAL 1      /* bad argument / unsupported block dims / misaligned frame size */
#define DCT3D_EDEVICE 2     /* no such HIP device, or a HIP runtime error */
#define DCT3D_ENOMEM 3      /* device or host allocation failed */
#define DCT3D_EKERNEL 4     /* a kernel launch failed */
#define DCT3D_ENOSPC 5      /* an output buffer is too small (nothing was written past its end) */
#define DCT3D_ENODATA 6     /* an input stream ends before the requested data is complete */

#define DCT3D_ABI_VERSION 8

typedef struct dct3d_ctx dct3d_ctx;

/* Per-call statistics of the certify-or-replay scheme (last encode/decode call on the ctx). */
typedef struct {
    uint64_t n_units;          /* coefficients (encode) or pixels (decode) produced by the last call */
    uint64_t n_flagged;        /* units of the last call re-done by the exact Java fold (decode: the 32
                                  pixels of every lane with an uncertified pixel) */
    /* HIP-event timing of every encode/decode call since dct3d_reset_timers (profiling on) */
    uint64_t n_timed;          /* calls timed */
    double kernel_ms_total;    /* main transform kernel, summed */
    double aux_ms_total;       /* the call's auxiliary launch, summed (fused Exp-Golomb encode: the
                                  compaction kernel); 0 for single-launch calls */
    uint64_t n_rechecked;      /* 8x8x8 encode: units of the last call the fp32 certificate left open
                                  and the fp64 second certificate settled (not counted in n_flagged) */
} dct3d_stats;

/* Transform-plan introspection (host only, no device needed). */
typedef struct {
    int cube_size;
    int n_mults;          /* sum over coefficients of Java multiplication groups (11,567 for 8^3) */
    int treeified;        /* 1 if Java's HashMap would have treeified a bin (fold order then unverified) */
    double coef_dc;       /* the single DC group coefficient (DCT.java:110 with k = 0) */
    double dec_G, dec_E;  /* decode certification: margin = L1 * dec_G + dec_E, L1 = sum |q * step| of the cube */
    float enc_rstep[32];  /* encode certification per s = kx+ky+kz: fp32(1/max(1,5s)) */
    float enc_G[32];      /*   threshold_s = 0.5 - (A * G_s + E_s), A = max|x - mean| of the cube */
    float enc_E[32];
    double enc_thr64[32]; /* 8x8x8 second certificate: settled iff |q64 - rint(q64)| < enc_thr64[s] */
    float dec_l1_max;     /* decode: a cube with L1 >= dec_l1_max takes the exact replay (|v| < 2^15) */
} dct3d_plan_info;

/* The plan for block dims (bw, bh, bd): the MI355X build's DCT.initialize (DCT.java:77-163) and
 * InverseDCT.initialize (InverseDCT.java:87-133).  Optional arrays (NULL to skip), cs = bw*bh*bd:
 *   ngroups [cs]       multiplication groups of each output coefficient k (fold length)
 *   coef    [cs * 64]  group coefficients of k in Java HashMap iteration (fold) order
 *   group_of[cs * cs]  fold index of input n in output k's fold (0xFF: dropped, key == 0)
 *   enc_K   [cs]       fp32 rounding-error bound of coefficient k per unit max|x - mean| */
int dct3d_plan_query(int bw, int bh, int bd, dct3d_plan_info *info, int32_t *ngroups, double *coef,
                     uint8_t *group_of, double *enc_K);

/* ABI version of the loaded library (DCT3D_ABI_VERSION). */
int dct3d_abi_version(void);
const char *dct3d_strerror(int code);

/* Replaces the per-call OpenCL setup: getDeviceId/getMaxWorkGroupSize (OpenCLUtils.c:69-104),
 * clCreateContext/buildKernel/clCreateBuffer/clCreateCommandQueue/clCreateKernel
 * (encoder.c:158-197, decoder.c:163-202).  `device` is a 0-based HIP ordinal (the codec layer
 * maps the reference's 1-based platformIndex, main.c:33-37).  Block dims are the codec.h macros
 * DCT_BLOCK_WIDTH/HEIGHT/DEPTH (codec.h:11-13); supported: 8 x 8 x 8 and 8 x 8 x 4. */
int dct3d_ctx_create(int device, int block_w, int block_h, int block_d, dct3d_ctx **out);
void dct3d_ctx_destroy(dct3d_ctx *ctx);

/* Use an external hipStream_t (e.g. a framework's current stream) instead of the ctx-owned one.
 * NULL restores the ctx-owned stream.  Work enqueued afterwards is ordered after the previous
 * stream's work by an event recorded on the previous stream, which therefore MUST STILL EXIST when
 * this is called: switch away from a caller's stream before destroying it.  (Should HIP reject the
 * previous handle, a device-wide synchronisation orders the work instead -- but a destroyed stream's
 * handle may already name a new stream, so that is no guarantee.) */
int dct3d_ctx_set_stream(dct3d_ctx *ctx, void *hip_stream);
/* The ctx's device ordinal, block depth and the hipStream_t its calls run on (any pointer may be
 * NULL).  Lets companion libraries (libdct3d_diag.so) queue work in order with the ctx's. */
int dct3d_ctx_info(const dct3d_ctx *ctx, int *device, int *block_d, void **hip_stream);
/* Test / diagnostic options of a ctx.  Each one changes only HOW later calls reach their results
 * (the results stay bit-identical): tests use them to drive the rare paths.  value 0 restores the
 * default.  Unknown options: DCT3D_EINVAL. */
#define DCT3D_OPT_DEC_MARGIN 2        /* added to the decode certification margin: lanes go to the in-wave
                                         exact replay */
#define DCT3D_OPT_ENC_NO_RECHECK 3    /* 1: the 8x8x8 encode skips its fp64 second certificate, so every
                                         coefficient the fp32 certificate leaves open takes the Java fold */
#define DCT3D_OPT_EG_TWO_STEP 5       /* 1: dct3d_encode_eg / dct3d_decode_eg through int32 cubes */
#define DCT3D_OPT_EG_NO_RESOLVE 6     /* 1: Exp-Golomb decode sync by plain confirming passes only */
#define DCT3D_OPT_EG_FORCE_RETRY 8    /* test: the Exp-Golomb decode's speculative front reports an unresolved
                                         pass 0, so the call takes its skip-and-rerun path (same results) */
#define DCT3D_OPT_EG_DEC_GROUPS 9     /* stream -> raster decode: groups of 2,048 values per wave, the next
                                         group's loads in flight during the current one (1, 2, 4, 8; 0: 8) */
#define DCT3D_OPT_EG_FUSED_FRONT 10   /* 1: the Exp-Golomb decode's speculative front as ONE launch (the
                                         resolving sync pass, the chunk scan and the mark pass fused, a
                                         decoupled look-back for the chunks' value indices) instead of three
                                         (A/B: measured slower) */
int dct3d_ctx_set_option(dct3d_ctx *ctx, int option, double value);
/* Enable HIP-event timing of the kernels (reported by dct3d_get_stats). */
int dct3d_ctx_set_profiling(dct3d_ctx *ctx, int on);
int dct3d_synchronize(dct3d_ctx *ctx);
/* Reads back the device counters of the last encode/decode and resolves the timing events
 * (synchronises the stream). */
int dct3d_get_stats(dct3d_ctx *ctx, dct3d_stats *out);
int dct3d_reset_timers(dct3d_ctx *ctx);

/* ---------------------------------------------------------------------------------------------
 * Native fused path (B): replaces readCubes + H2D + dct kernels + D2H + applyQuantization
 * (encoder.c:206-260) for n_stacks consecutive stacks.
 *   raster : n_stacks * block_d frames of width*height u8
 *   q_cubes: n_stacks * (width/bw) * (height/bh) cubes of bw*bh*bd int32 (cube-major)
 *   dct_opt: optional (may be NULL) fp64 DCT coefficients, same cube-major layout (the Java
 *            dctCoeff values, Encoder.java:66, for the float-DCT parity check)
 * ------------------------------------------------------------------------------------------- */
int dct3d_encode_stacks(dct3d_ctx *ctx, const uint8_t *raster, int width, int height, int n_stacks,
                        int32_t *q_cubes, double *dct_opt);
int dct3d_encode_stacks_dev(dct3d_ctx *ctx, const uint8_t *d_raster, int width, int height,
                            int n_stacks, int32_t *d_q_cubes, double *d_dct_opt);

/* Replaces applyDequantization + H2D + idct kernels + D2H + writeCubes (decoder.c:246-295). */
int dct3d_decode_stacks(dct3d_ctx *ctx, const int32_t *q_cubes, int width, int height, int n_stacks,
                        uint8_t *raster);
int dct3d_decode_stacks_dev(dct3d_ctx *ctx, const int32_t *d_q_cubes, int width, int height,
                            int n_stacks, uint8_t *d_raster);

/* ---------------------------------------------------------------------------------------------
 * Reference-faithful drop-in (A): the exact data flow of the OpenCL block, float cube-major in,
 * float cube-major out (kernelInputData -> kernelOutputData, encoder.c:165-254 / decoder.c:
 * 170-292).  The caller keeps readCubes/applyQuantization (forward) and applyDequantization/
 * writeCubes (inverse) on the host, exactly as the reference does.
 *   dct3d_forward_f32: orthonormal 3D DCT-II of each cube (dct_* kernels, 3dDCT.cl:43-143)
 *   dct3d_inverse_f32: 3D inverse DCT clamped to [0,255] (idct_* kernels, 3dDCT.cl:164-265)
 * ------------------------------------------------------------------------------------------- */
int dct3d_forward_f32(dct3d_ctx *ctx, const float *cubes, size_t n_cubes, float *coeffs);
int dct3d_inverse_f32(dct3d_ctx *ctx, const float *coeffs, size_t n_cubes, float *pixels);
int dct3d_forward_f32_dev(dct3d_ctx *ctx, const float *d_cubes, size_t n_cubes, float *d_coeffs);
int dct3d_inverse_f32_dev(dct3d_ctx *ctx, const float *d_coeffs, size_t n_cubes, float *d_pixels);

/* ---- Exp-Golomb stage on the device -----------------------------------------
 * Replaces applyExpGolombCoding (encoder.c:60-71) over expGolomb_writeValue (ExpGolomb.c:32-64) /
 * ExpGolombWriter.java:19-49: the signed order-0 Exp-Golomb stream of n_cubes consecutive cube-major
 * int32 cubes, each in diagonal-slice order (cubeUtils_diagonalSlices, CubeUtils.c:5-46), MSB first,
 * continuing a stream whose partial byte holds `carry_byte` with `carry_bits` (0..7) bits used (the
 * byte the reference carries from stack to stack, expGolomb_freeBuffer, ExpGolomb.c:112-130).
 * d_out (device, 4-byte aligned, out_cap bytes) receives ceil(total_bits / 32) little-endian words,
 * i.e. the stream bytes followed by zero padding; *total_bits = carry_bits + the bits written.
 * Values must satisfy |v| < 2^30 (quantised 8-bit content stays below 2^13), else DCT3D_EINVAL.
 * DCT3D_ENOSPC when out_cap is too small (*total_bits is still set; d_out is untouched).
 * Returns once *total_bits is known (the last kernel, eg_stitch_kernel, hands it to the host as it
 * starts); the last words of d_out complete on the context stream (dct3d_synchronize, or stream order). */
int dct3d_eg_encode_dev(dct3d_ctx *ctx, const int32_t *d_q, uint64_t n_cubes, uint8_t carry_byte, int carry_bits,
                        uint8_t *d_out, uint64_t out_cap, uint64_t *total_bits);

/* Host raster in, Exp-Golomb stream kept on the device: encoder.c:206-274 up to (not including) the
 * deflate -- readCubes + DCT + quantisation + applyExpGolombCoding for n_stacks stacks, one H2D copy
 * of the raw bytes.  *total_bits as above; fetch the bytes with dct3d_eg_fetch. */
int dct3d_encode_eg(dct3d_ctx *ctx, const uint8_t *raster, int width, int height, int n_stacks, uint8_t carry_byte,
                    int carry_bits, uint64_t *total_bits);

/* Device raster in, device stream out, fused: encoder.c:206-274 up to the deflate
 * (readCubes + DCT + quantisation + applyExpGolombCoding) for n_stacks stacks of d_raster, without
 * the int32 cube-major intermediate -- uncertified coefficients are replayed exactly inside the
 * transform kernel, and each wave codes its 8 cubes straight into the stream.  The stream format,
 * carry, d_out and *total_bits are those of dct3d_eg_encode_dev (the bytes are identical to
 * dct3d_encode_stacks_dev followed by dct3d_eg_encode_dev).  DCT3D_ENOSPC when out_cap is too small
 * (*total_bits is still set; d_out is untouched).  Returns as dct3d_eg_encode_dev: once *total_bits is
 * known, the last words completing on the context stream. */
int dct3d_encode_eg_dev(dct3d_ctx *ctx, const uint8_t *d_raster, int width, int height, int n_stacks,
                        uint8_t carry_byte, int carry_bits, uint8_t *d_out, uint64_t out_cap, uint64_t *total_bits);

/* Copies the first `nbytes` bytes of the last dct3d_encode_eg stream to host memory. */
int dct3d_eg_fetch(dct3d_ctx *ctx, uint8_t *out, uint64_t nbytes);

/* Diagonal-slice order of a bw x bh x bd cube (CubeUtils.c:5-46): out[i] = x + bw*y + bw*bh*z of the
 * i-th position (introspection / tests). */
int dct3d_diagonal_order(int bw, int bh, int bd, uint16_t *out);

/* Inverse of the Exp-Golomb stage (expGolomb_readValue, ExpGolomb.c:66-110 / ExpGolombReader.java;
 * Decoder.java:78-96 places value i of a cube at diagonal position i; decoder.c:210-236): decodes
 * n_cubes cubes (n_cubes * cube_size values) from the device stream d_bytes (4-byte aligned,
 * nbytes) starting at bit start_bit, into cube-major int32 d_q.  Parallel: self-synchronising
 * chunks of the stream (no index is needed in the file).  *end_bit = the bit after the last value.
 * DCT3D_ENODATA if the stream ends first, DCT3D_EINVAL if it is corrupt (a code with 32 or more
 * leading zeros).  Synchronises the context stream. */
int dct3d_eg_decode_dev(dct3d_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes, uint64_t start_bit, uint64_t n_cubes,
                        int32_t *d_q, uint64_t *end_bit);

/* Device stream in, device raster out, fused: decoder.c:209-295 after the inflate
 * for n_stacks stacks -- Exp-Golomb decode, reorder, dequantisation, IDCT, clamp/truncate -- without the
 * int32 cube-major intermediate: the decode kernel parses each of its cubes from the stream directly.
 * Stream arguments, *end_bit and errors as dct3d_eg_decode_dev; the raster as dct3d_decode_stacks_dev:
 * the call returns once *end_bit and the verdict are known (the decode kernel hands them to the host as
 * it starts), and the raster completes asynchronously on the context stream (use dct3d_synchronize, or
 * read it in stream order). */
int dct3d_decode_eg_dev(dct3d_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes, uint64_t start_bit, int width,
                        int height, int n_stacks, uint8_t *d_raster, uint64_t *end_bit);

/* Host stream in, raster out: decoder.c:209-295 after the inflate -- Exp-Golomb decode, reorder,
 * dequantisation, IDCT, clamp/truncate and writeCubes for n_stacks stacks, on the device; only the
 * stream and the u8 frames cross PCIe.  bytes[0..nbytes) holds the stream from bit start_bit (0..7). */
int dct3d_decode_eg(dct3d_ctx *ctx, const uint8_t *bytes, uint64_t nbytes, int start_bit, int width, int height,
                    int n_stacks, uint8_t *raster, uint64_t *end_bit);

#ifdef __cplusplus
}
#endif

#endif /* DCT3D_H_ */
