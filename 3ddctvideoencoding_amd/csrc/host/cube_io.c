/* cube_io.c -- reference-signature host helpers (encoder.c:10-58, decoder.c:10-72 semantics). */
#include "cube_io.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "codec.h"

size_t readCubes_d(FILE *in, float *data, int width, int height, int depth) {
    const size_t frame = (size_t)width * height, size = frame * depth;
    unsigned char *tmp = (unsigned char *)calloc(size, 1);  /* short stack -> zero-filled */
    if (!tmp) return 0;
    size_t got = 0, r;
    while (got < size && (r = fread(tmp + got, 1, size - got, in)) > 0) got += r;
    size_t o = 0;
    for (int y = 0; y < height; y += 8)
        for (int x = 0; x < width; x += 8)
            for (int k = 0; k < depth; k++)
                for (int i = 0; i < 8; i++)
                    for (int j = 0; j < 8; j++) data[o++] = tmp[k * frame + (size_t)(y + i) * width + x + j];
    free(tmp);
    return got;
}

size_t writeCubes_d(FILE *out, float *data, int width, int height, int depth) {
    const size_t frame = (size_t)width * height, size = frame * depth;
    unsigned char *tmp = (unsigned char *)malloc(size);
    if (!tmp) return 0;
    size_t o = 0;
    for (int y = 0; y < height; y += 8)
        for (int x = 0; x < width; x += 8)
            for (int k = 0; k < depth; k++)
                for (int i = 0; i < 8; i++)
                    for (int j = 0; j < 8; j++)
                        tmp[k * frame + (size_t)(y + i) * width + x + j] = (unsigned char)data[o++];
    size_t put = 0, w;
    while (put < size && (w = fwrite(tmp + put, 1, size - put, out)) > 0) put += w;
    free(tmp);
    return put;
}

void applyQuantization_d(float *c, size_t n, int depth) {
    const size_t cs = (size_t)64 * depth;
    for (size_t off = 0; off + cs <= n; off += cs)
        for (int z = 0; z < depth; z++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {
                    float *p = c + off + z * 64 + y * 8 + x;
                    *p = (float)round(*p / fmax(1, 5 * (x + y + z)));
                }
}

void applyDequantization_d(float *c, size_t n, int depth) {
    const size_t cs = (size_t)64 * depth;
    for (size_t off = 0; off + cs <= n; off += cs)
        for (int z = 0; z < depth; z++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {
                    float *p = c + off + z * 64 + y * 8 + x;
                    *p = (float)round(*p * fmax(1, 5 * (x + y + z)));
                }
}

void reorderDctCoeffs_d(float *c, size_t n, float *eg, struct SlicesPositions *sp, int depth) {
    const size_t cs = (size_t)64 * depth;
    size_t k = 0;
    for (size_t off = 0; off + cs <= n; off += cs)
        for (int i = 0; i < sp->length; i++) {
            const struct ThreeDimensionalCoordinates p = sp->positions[i];
            c[off + p.x + p.y * 8 + p.z * 64] = eg[k++];
        }
}

size_t readCubes(FILE *in, float *data, int width, int height) { return readCubes_d(in, data, width, height, DCT_BLOCK_DEPTH); }
size_t writeCubes(FILE *out, float *data, int width, int height) { return writeCubes_d(out, data, width, height, DCT_BLOCK_DEPTH); }
void applyQuantization(float *c, size_t n) { applyQuantization_d(c, n, DCT_BLOCK_DEPTH); }
void applyDequantization(float *c, size_t n) { applyDequantization_d(c, n, DCT_BLOCK_DEPTH); }
void reorderDctCoeffs(float *c, size_t n, float *eg, struct SlicesPositions *sp) {
    reorderDctCoeffs_d(c, n, eg, sp, DCT_BLOCK_DEPTH);
}
