/*
 * cube_io.h -- host-side cube pack/unpack and (de)quantisation helpers with the reference C codec's
 * signatures and semantics (encoder.c:10-58, decoder.c:10-72), kept for callers of the drop-in (A)
 * path (dct3d_forward_f32 / dct3d_inverse_f32).  The fused path (dct3d_encode_stacks /
 * dct3d_decode_stacks) does all of this on the device.
 *
 *   readCubes           u8 raster stack (fread) -> cube-major float           (encoder.c:10-45)
 *   writeCubes          cube-major float -> u8 raster ((unsigned char) cast)  (decoder.c:10-46)
 *   applyQuantization   c = round(c / fmax(1, 5(x+y+z))), C round() = half away from zero (encoder.c:47-58)
 *   applyDequantization c = round(c * fmax(1, 5(x+y+z)))                      (decoder.c:48-59)
 *   reorderDctCoeffs    diagonal-slice order -> cube-major                    (decoder.c:61-72)
 * The *_d variants take the block depth at run time; the plain ones use DCT_BLOCK_DEPTH.
 * readCubes zero-fills a short last stack (the reference leaves uninitialised bytes there).
 */
#ifndef DCT3D_CUBE_IO_H_
#define DCT3D_CUBE_IO_H_

#include <stddef.h>
#include <stdio.h>

#include "cube_utils.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Difference from the reference: readCubes / writeCubes return size_t where the reference returns
 * void (encoder.c:10, decoder.c:10).  readCubes returns the number of raw bytes actually read
 * (< width*height*depth at end of file), writeCubes the number of bytes written.  A caller written
 * against the reference's prototypes (ignoring the result) compiles and links unchanged: on every
 * C ABI in use the return register is simply not read, and no argument changes. */
size_t readCubes(FILE *inputFile, float *data, int width, int height);
size_t writeCubes(FILE *outputFile, float *data, int width, int height);
void applyQuantization(float *dctCoeff, size_t bufferSize);
void applyDequantization(float *dctCoeff, size_t bufferSize);
void reorderDctCoeffs(float *dctCoeff, size_t bufferSize, float *expGolombDecodedData,
                      struct SlicesPositions *slicesPositions);

size_t readCubes_d(FILE *inputFile, float *data, int width, int height, int depth);
size_t writeCubes_d(FILE *outputFile, float *data, int width, int height, int depth);
void applyQuantization_d(float *dctCoeff, size_t bufferSize, int depth);
void applyDequantization_d(float *dctCoeff, size_t bufferSize, int depth);
void reorderDctCoeffs_d(float *dctCoeff, size_t bufferSize, float *expGolombDecodedData,
                        struct SlicesPositions *slicesPositions, int depth);

#ifdef __cplusplus
}
#endif

#endif
