/*
 * codec.h -- reference-compatible codec entry points and block dimensions
 * (replaces 3d-DCT-video-encoding-OpenCL/codec.h:11-20).
 *
 * Same macro names as the reference; FACE_SIZE / CUBE_SIZE are parenthesised here (the reference's
 * unparenthesised `#define CUBE_SIZE FACE_SIZE * DCT_BLOCK_DEPTH` silently breaks `x / CUBE_SIZE`).
 * DCT_BLOCK_DEPTH may be overridden at compile time (8 or 4); the *_ex entry points
 * take it at run time.
 */
#ifndef DCT3D_CODEC_H_
#define DCT3D_CODEC_H_

#define DCT_BLOCK_WIDTH 8
#define DCT_BLOCK_HEIGHT 8
#ifndef DCT_BLOCK_DEPTH
#define DCT_BLOCK_DEPTH 8
#endif

#define FACE_SIZE (DCT_BLOCK_WIDTH * DCT_BLOCK_HEIGHT)
#define CUBE_SIZE (FACE_SIZE * DCT_BLOCK_DEPTH)

#ifdef __cplusplus
extern "C" {
#endif

/* encoder.c:88 / decoder.c:85.  platformIndex is the reference's 1-based device selector
 * (main.c:33-37); here it selects HIP device (platformIndex - 1).  Returns 0 on success, 1 on
 * failure after printing the reason (the reference's convention). */
int encode(char *inputFileName, char *outputFileName, int width, int height, int framesToEncode, int platformIndex);
int decode(char *inputFileName, char *outputFileName, int width, int height, int framesToDecode, int platformIndex);

/* Same, with the block depth (8 or 4) and the number of stacks per device call explicit. */
int encode_ex(const char *inputFileName, const char *outputFileName, int width, int height, int framesToEncode,
              int platformIndex, int blockDepth, int stacksPerBatch);
int decode_ex(const char *inputFileName, const char *outputFileName, int width, int height, int framesToDecode,
              int platformIndex, int blockDepth, int stacksPerBatch);

/* Several devices (platformIndices[0 .. nDevices-1], 1-based; a device may repeat), one host thread and
 * one context each.  encode_multi: batches round-robin over the devices, their streams joined in order:
 * the same .bin as encode_ex.  decode_multi: the batches' device decodes chain on the stream position
 * (the stream has no index) and alternate over the devices; only the previous batch's raster write
 * overlaps a decode (with two or more devices), so decoding does not scale with devices.  Same return
 * convention. */
int encode_multi(const char *inputFileName, const char *outputFileName, int width, int height, int framesToEncode,
                 const int *platformIndices, int nDevices, int blockDepth, int stacksPerBatch);
int decode_multi(const char *inputFileName, const char *outputFileName, int width, int height, int framesToDecode,
                 const int *platformIndices, int nDevices, int blockDepth, int stacksPerBatch);

#ifdef __cplusplus
}
#endif

#endif /* DCT3D_CODEC_H_ */
