/* exp_golomb.c -- signed order-0 Exp-Golomb stream.  Byte-identical to the reference writers
 * (ExpGolomb.c:32-64, ExpGolombWriter.java:19-49) on a zeroed buffer, same reader semantics
 * (ExpGolomb.c:66-110, ExpGolombReader.java:19-63).  The stream is a plain MSB-first concatenation
 * of codewords: bufferPosition = bits/8, bitPosition = 8 - bits%8. */
#include "exp_golomb.h"

#include <stdlib.h>
#include <string.h>

struct ExpGolombStream *expGolomb_createStream(char *buffer) {
    struct ExpGolombStream *s = (struct ExpGolombStream *)malloc(sizeof(*s));
    if (!s) return NULL;
    s->buffer = buffer;
    s->bitPosition = 8;
    s->bufferPosition = 0;
    if (buffer) buffer[0] = 0;
    return s;
}

void expGolomb_destroyStream(struct ExpGolombStream *s) { free(s); }

static unsigned eg_code(int value, int *nbits) {
    unsigned v = value <= 0 ? (unsigned)(-2 * (long long)value) : (unsigned)(2 * (long long)value - 1);
    v += 1;
    int n = 0;
    for (unsigned t = v; t; t >>= 1) n++;
    *nbits = n;
    return v;
}

/* appends `count` bits (MSB first) of `bits` at the stream cursor */
static void put_bits(struct ExpGolombStream *s, unsigned bits, int count) {
    while (count > 0) {
        const int take = count < s->bitPosition ? count : s->bitPosition;
        const unsigned chunk = (bits >> (count - take)) & ((1u << take) - 1u);
        s->buffer[s->bufferPosition] = (char)((unsigned char)s->buffer[s->bufferPosition] | (chunk << (s->bitPosition - take)));
        s->bitPosition -= take;
        count -= take;
        if (s->bitPosition == 0) {
            s->bufferPosition++;
            s->bitPosition = 8;
            s->buffer[s->bufferPosition] = 0;
        }
    }
}

void expGolomb_writeValue(struct ExpGolombStream *s, int value) {
    int n;
    const unsigned v = eg_code(value, &n);
    /* n-1 zero bits, then the n-bit value */
    int zeros = n - 1;
    while (zeros > 0) {
        const int take = zeros < s->bitPosition ? zeros : s->bitPosition;
        s->bitPosition -= take;
        zeros -= take;
        if (s->bitPosition == 0) {
            s->bufferPosition++;
            s->bitPosition = 8;
            s->buffer[s->bufferPosition] = 0;
        }
    }
    put_bits(s, v, n);
}

static int get_bit(struct ExpGolombStream *s) {
    const int bit = ((unsigned char)s->buffer[s->bufferPosition] >> (s->bitPosition - 1)) & 1;
    if (--s->bitPosition == 0) {
        s->bitPosition = 8;
        s->bufferPosition++;
    }
    return bit;
}

int expGolomb_readValue(struct ExpGolombStream *s) {
    int zeros = 0;
    while (get_bit(s) == 0) zeros++;
    unsigned v = 1;
    for (int i = 0; i < zeros; i++) v = (v << 1) | (unsigned)get_bit(s);
    long long value = (long long)v - 1;
    return (value % 2 != 0) ? (int)((value + 1) / 2) : (int)(-value / 2);
}

void expGolomb_freeBuffer(struct ExpGolombStream *s, int position, int writing) {
    if (writing) {
        if (position <= s->bufferPosition) {
            memmove(s->buffer, s->buffer + position, (size_t)(s->bufferPosition - position + 1));
            s->bufferPosition -= position;
        } else {
            s->bufferPosition = 0;
            s->buffer[0] = 0;
        }
    } else {
        if (position > s->bufferPosition)
            memmove(s->buffer, s->buffer + s->bufferPosition, (size_t)(position - s->bufferPosition));
        s->bufferPosition = 0;
    }
}
