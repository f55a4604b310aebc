/* codec.c -- encode()/decode(): the reference codec's pipeline (encoder.c:88-293,
 * decoder.c:85-314) with the OpenCL block replaced by the libdct3d C-ABI.
 *
 * encode: per batch of stacks: fread -> dct3d_encode_stacks (fused DCT + quantisation on the GPU,
 *         Java semantics) -> per stack: diagonal order + Exp-Golomb + deflate (codec_entropy.c).
 * decode: inflate + Exp-Golomb + reorder per stack -> dct3d_decode_stacks (fused dequantisation +
 *         IDCT + clamp + truncation on the GPU) -> fwrite.
 * A stack is DCT_BLOCK_DEPTH frames; a short last stack is zero-filled (the reference reads
 * uninitialised bytes there, encoder.c:21-27).  Frames to encode are rounded up to whole stacks,
 * as in the reference loop (encoder.c:203).  Errors: printf + return 1 (the reference convention);
 * never exit(). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "codec.h"
#include "codec_entropy.h"
#include "dct3d.h"

static int default_batch(void) {
    const char *e = getenv("DCT3D_CODEC_BATCH");
    int b = e ? atoi(e) : 16;
    return b > 0 ? b : 16;
}

int encode_ex(const char *inName, const char *outName, int width, int height, int frames, int platformIndex,
              int depth, int batch) {
    if (width <= 0 || height <= 0 || width % 8 || height % 8 || frames <= 0 || (depth != 8 && depth != 4)) {
        printf("Invalid geometry: %dx%d, %d frames, block depth %d (width/height must be multiples of 8)\n", width,
               height, frames, depth);
        return 1;
    }
    if (batch <= 0) batch = default_batch();
    FILE *in = fopen(inName, "rb");
    if (!in) {
        printf("Cannot open input file %s\n", inName);
        return 1;
    }
    FILE *out = fopen(outName, "wb");
    if (!out) {
        printf("Cannot open output file %s\n", outName);
        fclose(in);
        return 1;
    }
    dct3d_ctx *ctx = NULL;
    int rc = dct3d_ctx_create(platformIndex > 0 ? platformIndex - 1 : 0, 8, 8, depth, &ctx);
    if (rc) {
        printf("Error creating the device context: %s\n", dct3d_strerror(rc));
        fclose(in);
        fclose(out);
        return 1;
    }
    const size_t frame = (size_t)width * height, stack_px = frame * depth;
    const int n_stacks = (frames + depth - 1) / depth;
    /* DCT3D_CODEC_HOST_EG=1: Exp-Golomb on the host from the quantised ints (A/B and tests); default:
     * the device Exp-Golomb stage, the same bytes */
    const char *he = getenv("DCT3D_CODEC_HOST_EG");
    const int host_eg = he && he[0] == '1';
    uint8_t *raster = (uint8_t *)malloc(stack_px * batch);
    int32_t *q = host_eg ? (int32_t *)malloc(stack_px * batch * sizeof(int32_t)) : NULL;
    size_t eg_cap = stack_px * batch / 2 + 64;
    unsigned char *eg = host_eg ? NULL : (unsigned char *)malloc(eg_cap);
    dct3d_entropy_enc *ent = dct3d_entropy_enc_create(width, height, depth, out);
    /* DCT3D_CODEC_DEFLATE_THREADS=N (N > 1): parallel deflate -- the same inflated payload, a different
     * .bin; default: one zlib stream, the reference encoder's bytes */
    const char *dt = getenv("DCT3D_CODEC_DEFLATE_THREADS");
    const int deflate_threads = dt ? atoi(dt) : 1;
    int status = 0;
    if (ent && dct3d_entropy_enc_set_threads(ent, deflate_threads, 0)) {
        dct3d_entropy_enc_destroy(ent);
        ent = NULL;
    }
    if (!raster || (host_eg ? !q : !eg) || !ent) {
        printf("Out of memory\n");
        status = 1;
    }
    for (int s0 = 0; !status && s0 < n_stacks; s0 += batch) {
        const int nb = (n_stacks - s0) < batch ? (n_stacks - s0) : batch;
        size_t got = 0, r;
        const size_t want = stack_px * nb;
        while (got < want && (r = fread(raster + got, 1, want - got, in)) > 0) got += r;
        if (got < want) memset(raster + got, 0, want - got);
        const int last = s0 + nb == n_stacks;
        if (host_eg) {  /* quantised ints over PCIe, Exp-Golomb on the host (the reference's split) */
            rc = dct3d_encode_stacks(ctx, raster, width, height, nb, q, NULL);
            if (rc) {
                printf("Error running the 3D DCT: %s\n", dct3d_strerror(rc));
                status = 1;
                break;
            }
            for (int s = 0; s < nb; s++) {
                if (dct3d_entropy_enc_push(ent, q + stack_px * s, s0 + s == n_stacks - 1)) {
                    printf("Error in the entropy coder\n");
                    status = 1;
                    break;
                }
            }
        } else {  /* DCT + quantisation + diagonal order + Exp-Golomb on the device; the stream over PCIe */
            uint8_t cb;
            int cbits;
            uint64_t tb = 0;
            dct3d_entropy_enc_carry(ent, &cb, &cbits);
            rc = dct3d_encode_eg(ctx, raster, width, height, nb, cb, cbits, &tb);
            const size_t nbytes = (size_t)((tb + 7) / 8);
            if (!rc && nbytes > eg_cap) {
                free(eg);
                eg_cap = nbytes + nbytes / 4;
                eg = (unsigned char *)malloc(eg_cap);
                if (!eg) rc = DCT3D_ENOMEM;
            }
            if (!rc) rc = dct3d_eg_fetch(ctx, eg, nbytes);
            if (rc) {
                printf("Error running the 3D DCT: %s\n", dct3d_strerror(rc));
                status = 1;
                break;
            }
            if (dct3d_entropy_enc_push_stream(ent, eg, tb, last)) {
                printf("Error in the entropy coder\n");
                status = 1;
                break;
            }
        }
        for (int s = 0; !status && s < nb; s++) printf("Frames processed: %d\n", (s0 + s + 1) * depth);
    }
    dct3d_entropy_enc_destroy(ent);
    free(raster);
    free(q);
    free(eg);
    dct3d_ctx_destroy(ctx);
    fclose(in);
    if (fflush(out) || fclose(out)) status = 1;
    if (!status) printf("Encoding process completed\n");
    return status;
}

int decode_ex(const char *inName, const char *outName, int width, int height, int frames, int platformIndex,
              int depth, int batch) {
    if (width <= 0 || height <= 0 || width % 8 || height % 8 || frames <= 0 || (depth != 8 && depth != 4)) {
        printf("Invalid geometry: %dx%d, %d frames, block depth %d\n", width, height, frames, depth);
        return 1;
    }
    if (batch <= 0) batch = default_batch();
    FILE *in = fopen(inName, "rb");
    if (!in) {
        printf("Cannot open input file %s\n", inName);
        return 1;
    }
    FILE *out = fopen(outName, "wb");
    if (!out) {
        printf("Cannot open output file %s\n", outName);
        fclose(in);
        return 1;
    }
    dct3d_ctx *ctx = NULL;
    int rc = dct3d_ctx_create(platformIndex > 0 ? platformIndex - 1 : 0, 8, 8, depth, &ctx);
    if (rc) {
        printf("Error creating the device context: %s\n", dct3d_strerror(rc));
        fclose(in);
        fclose(out);
        return 1;
    }
    const size_t frame = (size_t)width * height, stack_px = frame * depth;
    const int n_stacks = (frames + depth - 1) / depth;
    /* DCT3D_CODEC_HOST_EG=1: Exp-Golomb decode on the host, ints over PCIe (the reference's split);
     * default: the device decodes the inflated stream (dct3d_decode_eg), only the stream crosses PCIe */
    const char *he = getenv("DCT3D_CODEC_HOST_EG");
    const int host_eg = he && he[0] == '1';
    uint8_t *raster = (uint8_t *)malloc(stack_px * batch);
    int32_t *q = host_eg ? (int32_t *)malloc(stack_px * batch * sizeof(int32_t)) : NULL;
    dct3d_entropy_dec *ent = dct3d_entropy_dec_create(width, height, depth, in, NULL, 0);
    int status = 0;
    double bits_per_value = 4.0;  /* window estimate for the first batch; then the measured rate */
    if (!raster || (host_eg && !q) || !ent) {
        printf("Out of memory\n");
        status = 1;
    }
    for (int s0 = 0; !status && s0 < n_stacks; s0 += batch) {
        const int nb = (n_stacks - s0) < batch ? (n_stacks - s0) : batch;
        if (host_eg) {
            for (int s = 0; s < nb; s++)
                if (dct3d_entropy_dec_pull(ent, q + stack_px * s)) {
                    printf("Truncated or corrupt input stream\n");
                    status = 1;
                    break;
                }
            if (status) break;
            rc = dct3d_decode_stacks(ctx, q, width, height, nb, raster);
        } else {
            const double values = (double)stack_px * nb;
            size_t need = (size_t)(values * bits_per_value / 8 * 1.25) + 65536;
            for (;;) {
                const unsigned char *p;
                size_t len;
                int bit;
                uint64_t eb = 0;
                if (dct3d_entropy_dec_window(ent, need, &p, &len, &bit)) {
                    rc = DCT3D_EINVAL;
                    break;
                }
                rc = dct3d_decode_eg(ctx, p, len, bit, width, height, nb, raster, &eb);
                if (rc == DCT3D_ENODATA && !dct3d_entropy_dec_eof(ent) && len >= need) {
                    need *= 2;  /* the batch needs more of the stream than estimated */
                    continue;
                }
                if (!rc) {
                    dct3d_entropy_dec_consume(ent, eb);
                    bits_per_value = (double)(eb - (uint64_t)bit) / values;
                }
                break;
            }
            if (rc == DCT3D_ENODATA || rc == DCT3D_EINVAL) {
                printf("Truncated or corrupt input stream\n");
                status = 1;
                break;
            }
        }
        if (rc) {
            printf("Error running the inverse 3D DCT: %s\n", dct3d_strerror(rc));
            status = 1;
            break;
        }
        if (fwrite(raster, 1, stack_px * nb, out) != stack_px * nb) {
            printf("Error writing the output file\n");
            status = 1;
            break;
        }
        printf("Frames processed: %d\n", (s0 + nb) * depth);
    }
    dct3d_entropy_dec_destroy(ent);
    free(raster);
    free(q);
    dct3d_ctx_destroy(ctx);
    fclose(in);
    if (fflush(out) || fclose(out)) status = 1;
    if (!status) printf("Decoding process completed\n");
    return status;
}

int encode(char *inName, char *outName, int width, int height, int frames, int platformIndex) {
    return encode_ex(inName, outName, width, height, frames, platformIndex, DCT_BLOCK_DEPTH, 0);
}

int decode(char *inName, char *outName, int width, int height, int frames, int platformIndex) {
    return decode_ex(inName, outName, width, height, frames, platformIndex, DCT_BLOCK_DEPTH, 0);
}
