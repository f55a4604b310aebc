/*
 * exp_golomb.h -- signed order-0 Exp-Golomb bit stream
 * (replaces 3d-DCT-video-encoding-OpenCL/ExpGolomb.h:4-16; Java ExpGolombWriter/Reader.java).
 * Mapping v <= 0 -> -2v, v > 0 -> 2v - 1, then +1, MSB first.  bitPosition counts the free bits of
 * the current byte (8 = empty).  Unlike the reference, createStream zeroes the first byte (the
 * reference ORs into an uninitialised malloc'd byte, ExpGolomb.c:24-30 + encoder.c:133).
 */
#ifndef DCT3D_EXP_GOLOMB_H_
#define DCT3D_EXP_GOLOMB_H_

#ifdef __cplusplus
extern "C" {
#endif

struct ExpGolombStream {
    char *buffer;
    int bitPosition;
    int bufferPosition;
};

struct ExpGolombStream *expGolomb_createStream(char *buffer);
void expGolomb_writeValue(struct ExpGolombStream *stream, int value);
int expGolomb_readValue(struct ExpGolombStream *stream);
/* writing: keep the partial byte at `position` (moves it to the front); reading: drop the consumed
 * bytes [0, bufferPosition) of a buffer holding `position` valid bytes (ExpGolomb.c:112-130). */
void expGolomb_freeBuffer(struct ExpGolombStream *stream, int position, int writing);
void expGolomb_destroyStream(struct ExpGolombStream *stream);

#ifdef __cplusplus
}
#endif

#endif
