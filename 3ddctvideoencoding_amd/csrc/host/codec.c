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
 * never exit().
 *
 * encode_multi / decode_multi: the same pipelines over several devices, one host thread and one
 * dct3d_ctx per device (a ctx is single-threaded; SURVEY.md §8b "one host thread per ctx").  Encode:
 * batches go round-robin to the devices, each coded from a zero carry; the calling thread joins the
 * batch streams in order, shifting each by the running partial byte, into the one zlib stream -- the
 * same .bin as encode_ex.  Decode: a batch's first bit is known only when the previous batch is
 * decoded (the stream has no index), so the device calls chain and alternate over the devices; the only
 * overlap is the previous batch's raster write (several devices) -- the next window is inflated after
 * the running decode returns.  Decoding does not get faster with more devices. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "codec.h"
#include "codec_entropy.h"
#include "dct3d.h"

/* DCT3D_CODEC_TIMING=1: encode_ex / decode_ex print one JSON line of per-stage wall seconds to stderr
 * (tools/codec_e2e.py): which stage bounds the reference-identical .bin end to end */
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
static int timing_on(void) {
    const char *e = getenv("DCT3D_CODEC_TIMING");
    return e && e[0] == '1';
}
#define STAGE(acc, stmt)              \
    do {                              \
        const double t_0_ = now_s();  \
        stmt;                         \
        (acc) += now_s() - t_0_;      \
    } while (0)

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
    const double t_start = now_s();
    double t_read = 0, t_dev = 0, t_fetch = 0, t_ent = 0;
    int rc = dct3d_ctx_create(platformIndex > 0 ? platformIndex - 1 : 0, 8, 8, depth, &ctx);
    const double t_ctx = now_s() - t_start;
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
        STAGE(t_read, while (got < want && (r = fread(raster + got, 1, want - got, in)) > 0) got += r);
        if (got < want) memset(raster + got, 0, want - got);
        const int last = s0 + nb == n_stacks;
        if (host_eg) {  /* quantised ints over PCIe, Exp-Golomb on the host (the reference's split) */
            STAGE(t_dev, rc = dct3d_encode_stacks(ctx, raster, width, height, nb, q, NULL));
            if (rc) {
                printf("Error running the 3D DCT: %s\n", dct3d_strerror(rc));
                status = 1;
                break;
            }
            const double t_e0 = now_s();
            for (int s = 0; s < nb; s++) {
                if (dct3d_entropy_enc_push(ent, q + stack_px * s, s0 + s == n_stacks - 1)) {
                    printf("Error in the entropy coder\n");
                    status = 1;
                    break;
                }
            }
            t_ent += now_s() - t_e0;
        } else {  /* DCT + quantisation + diagonal order + Exp-Golomb on the device; the stream over PCIe */
            uint8_t cb;
            int cbits;
            uint64_t tb = 0;
            dct3d_entropy_enc_carry(ent, &cb, &cbits);
            STAGE(t_dev, rc = dct3d_encode_eg(ctx, raster, width, height, nb, cb, cbits, &tb));
            const size_t nbytes = (size_t)((tb + 7) / 8);
            if (!rc && nbytes > eg_cap) {
                free(eg);
                eg_cap = nbytes + nbytes / 4;
                eg = (unsigned char *)malloc(eg_cap);
                if (!eg) rc = DCT3D_ENOMEM;
            }
            if (!rc) STAGE(t_fetch, rc = dct3d_eg_fetch(ctx, eg, nbytes));
            if (rc) {
                printf("Error running the 3D DCT: %s\n", dct3d_strerror(rc));
                status = 1;
                break;
            }
            int perr;
            STAGE(t_ent, perr = dct3d_entropy_enc_push_stream(ent, eg, tb, last));
            if (perr) {
                printf("Error in the entropy coder\n");
                status = 1;
                break;
            }
        }
        for (int s = 0; !status && s < nb; s++) printf("Frames processed: %d\n", (s0 + s + 1) * depth);
    }
    STAGE(t_ent, dct3d_entropy_enc_destroy(ent));  /* the last deflate output and its write */
    free(raster);
    free(q);
    free(eg);
    dct3d_ctx_destroy(ctx);
    fclose(in);
    if (fflush(out) || fclose(out)) status = 1;
    if (timing_on())
        fprintf(stderr,
                "{\"stage_s\": {\"ctx_create\": %.6f, \"read\": %.6f, \"device\": %.6f, \"eg_fetch\": %.6f, "
                "\"%s\": %.6f}, \"total_s\": %.6f, \"host_eg\": %d, \"deflate_threads\": %d}\n",
                t_ctx, t_read, t_dev, t_fetch, host_eg ? "eg_deflate_write" : "deflate_write", t_ent, now_s() - t_start,
                host_eg, deflate_threads);
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
    const double t_start = now_s();
    double t_inf = 0, t_dev = 0, t_write = 0;
    int rc = dct3d_ctx_create(platformIndex > 0 ? platformIndex - 1 : 0, 8, 8, depth, &ctx);
    const double t_ctx = now_s() - t_start;
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
            const double t_i0 = now_s();
            for (int s = 0; s < nb; s++)
                if (dct3d_entropy_dec_pull(ent, q + stack_px * s)) {
                    printf("Truncated or corrupt input stream\n");
                    status = 1;
                    break;
                }
            t_inf += now_s() - t_i0;
            if (status) break;
            STAGE(t_dev, rc = dct3d_decode_stacks(ctx, q, width, height, nb, raster));
        } else {
            const double values = (double)stack_px * nb;
            size_t need = (size_t)(values * bits_per_value / 8 * 1.25) + 65536;
            for (;;) {
                const unsigned char *p;
                size_t len;
                int bit;
                uint64_t eb = 0;
                int werr;
                STAGE(t_inf, werr = dct3d_entropy_dec_window(ent, need, &p, &len, &bit));
                if (werr) {
                    rc = DCT3D_EINVAL;
                    break;
                }
                STAGE(t_dev, rc = dct3d_decode_eg(ctx, p, len, bit, width, height, nb, raster, &eb));
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
        size_t wrote;
        STAGE(t_write, wrote = fwrite(raster, 1, stack_px * nb, out));
        if (wrote != stack_px * nb) {
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
    STAGE(t_write, if (fflush(out) || fclose(out)) status = 1);
    if (timing_on())
        fprintf(stderr,
                "{\"stage_s\": {\"ctx_create\": %.6f, \"%s\": %.6f, \"device\": %.6f, \"write\": %.6f}, "
                "\"total_s\": %.6f, \"host_eg\": %d}\n",
                t_ctx, host_eg ? "read_inflate_eg" : "read_inflate", t_inf, t_dev, t_write, now_s() - t_start, host_eg);
    if (!status) printf("Decoding process completed\n");
    return status;
}

/* ---- several devices ------------------------------------------------------------------------ */

typedef struct {
    dct3d_ctx *ctx;
    int width, height, decode;
    pthread_t th;
    int started;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int state;  /* 0 idle, 1 job posted, 2 job done, 3 quit */
    int rc;
    int nb;                 /* stacks of the job */
    uint8_t *raster;        /* encode: input; decode: output (stack_px * batch) */
    unsigned char *eg;      /* encode: the batch's stream, fetched (grown as needed) */
    size_t eg_cap;
    uint64_t bits;          /* encode: stream bits; decode: bits consumed from the window */
    const unsigned char *win;  /* decode: the inflated window, its length and first bit */
    size_t win_len;
    int win_bit;
} dev_worker;

static void *dev_worker_main(void *arg) {
    dev_worker *w = (dev_worker *)arg;
    for (;;) {
        pthread_mutex_lock(&w->mu);
        while (w->state != 1 && w->state != 3) pthread_cond_wait(&w->cv, &w->mu);
        const int quit = w->state == 3;
        pthread_mutex_unlock(&w->mu);
        if (quit) return NULL;
        int rc;
        if (!w->decode) {
            uint64_t tb = 0;
            rc = dct3d_encode_eg(w->ctx, w->raster, w->width, w->height, w->nb, 0, 0, &tb);
            const size_t nbytes = (size_t)((tb + 7) / 8);
            if (!rc && nbytes > w->eg_cap) {
                free(w->eg);
                w->eg_cap = nbytes + nbytes / 4;
                w->eg = (unsigned char *)malloc(w->eg_cap);
                if (!w->eg) rc = DCT3D_ENOMEM;
            }
            if (!rc) rc = dct3d_eg_fetch(w->ctx, w->eg, nbytes);
            w->bits = tb;
        } else {
            uint64_t eb = 0;
            rc = dct3d_decode_eg(w->ctx, w->win, w->win_len, w->win_bit, w->width, w->height, w->nb, w->raster, &eb);
            w->bits = eb;
        }
        pthread_mutex_lock(&w->mu);
        w->rc = rc;
        w->state = 2;
        pthread_cond_broadcast(&w->cv);
        pthread_mutex_unlock(&w->mu);
    }
}

static void dev_post(dev_worker *w) {
    pthread_mutex_lock(&w->mu);
    w->state = 1;
    pthread_cond_broadcast(&w->cv);
    pthread_mutex_unlock(&w->mu);
}

static int dev_wait(dev_worker *w) {
    pthread_mutex_lock(&w->mu);
    while (w->state != 2) pthread_cond_wait(&w->cv, &w->mu);
    w->state = 0;
    const int rc = w->rc;
    pthread_mutex_unlock(&w->mu);
    return rc;
}

static void dev_workers_destroy(dev_worker *ws, int n) {
    if (!ws) return;
    for (int i = 0; i < n; i++) {
        dev_worker *w = &ws[i];
        if (w->started) {
            pthread_mutex_lock(&w->mu);
            while (w->state == 1) pthread_cond_wait(&w->cv, &w->mu);  /* a posted job finishes first */
            w->state = 3;
            pthread_cond_broadcast(&w->cv);
            pthread_mutex_unlock(&w->mu);
            pthread_join(w->th, NULL);
            pthread_mutex_destroy(&w->mu);
            pthread_cond_destroy(&w->cv);
        }
        dct3d_ctx_destroy(w->ctx);
        free(w->raster);
        free(w->eg);
    }
    free(ws);
}

/* one ctx + thread per device (platform indices 1-based, as encode_ex); NULL after printing on failure */
static dev_worker *dev_workers_create(const int *platformIndices, int n, int width, int height, int depth,
                                      size_t raster_bytes, int decode) {
    dev_worker *ws = (dev_worker *)calloc((size_t)n, sizeof(dev_worker));
    if (!ws) {
        printf("Out of memory\n");
        return NULL;
    }
    for (int i = 0; i < n; i++) {
        dev_worker *w = &ws[i];
        w->width = width;
        w->height = height;
        w->decode = decode;
        const int idx = platformIndices[i];
        int rc = dct3d_ctx_create(idx > 0 ? idx - 1 : 0, 8, 8, depth, &w->ctx);
        if (rc) {
            printf("Error creating the device context (device %d): %s\n", idx, dct3d_strerror(rc));
            dev_workers_destroy(ws, n);
            return NULL;
        }
        w->raster = (uint8_t *)malloc(raster_bytes);
        if (!w->raster || pthread_mutex_init(&w->mu, NULL) || pthread_cond_init(&w->cv, NULL)) {
            printf("Out of memory\n");
            dev_workers_destroy(ws, n);
            return NULL;
        }
        if (pthread_create(&w->th, NULL, dev_worker_main, w)) {
            pthread_mutex_destroy(&w->mu);
            pthread_cond_destroy(&w->cv);
            printf("Cannot start a device thread\n");
            dev_workers_destroy(ws, n);
            return NULL;
        }
        w->started = 1;
    }
    return ws;
}

/* `bits` stream bits coded from a zero carry, re-aligned behind the c (0..7) bits of the partial byte
 * cb (MSB first): out[0] = cb | s[0] >> c, out[i] = s[i-1] << (8 - c) | s[i] >> c; returns the bits */
static uint64_t join_carry(const unsigned char *s, uint64_t bits, uint8_t cb, int c, unsigned char *out) {
    const size_t n = (size_t)((bits + 7) / 8), m = (size_t)((bits + (uint64_t)c + 7) / 8);
    if (c == 0) {
        memcpy(out, s, n);
        return bits;
    }
    unsigned prev = cb >> (8 - c);
    for (size_t i = 0; i < m; i++) {
        const unsigned cur = i < n ? s[i] : 0u;
        out[i] = (unsigned char)((prev << (8 - c)) | (cur >> c));
        prev = cur;
    }
    return bits + (uint64_t)c;
}

int encode_multi(const char *inName, const char *outName, int width, int height, int frames,
                 const int *platformIndices, int nDevices, int depth, int batch) {
    if (!platformIndices || nDevices <= 0) {
        printf("No device given\n");
        return 1;
    }
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
    const size_t frame = (size_t)width * height, stack_px = frame * depth;
    const int n_stacks = (frames + depth - 1) / depth;
    const int n_batches = (n_stacks + batch - 1) / batch;
    dev_worker *ws = dev_workers_create(platformIndices, nDevices, width, height, depth, stack_px * batch, 0);
    if (!ws) {
        fclose(in);
        fclose(out);
        return 1;
    }
    dct3d_entropy_enc *ent = dct3d_entropy_enc_create(width, height, depth, out);
    const char *dt = getenv("DCT3D_CODEC_DEFLATE_THREADS");
    int status = 0;
    if (ent && dct3d_entropy_enc_set_threads(ent, dt ? atoi(dt) : 1, 0)) {
        dct3d_entropy_enc_destroy(ent);
        ent = NULL;
    }
    unsigned char *joined = NULL;
    size_t joined_cap = 0;
    if (!ent) {
        printf("Out of memory\n");
        status = 1;
    }
    /* batch k runs on device k % n; up to n batches in flight, joined in order */
    int posted = 0;
    for (int k = 0; !status && k < n_batches; k++) {
        for (; posted < n_batches && posted < k + nDevices; posted++) {
            dev_worker *w = &ws[posted % nDevices];
            const int s0 = posted * batch, nb = (n_stacks - s0) < batch ? (n_stacks - s0) : batch;
            size_t got = 0, r;
            const size_t want = stack_px * (size_t)nb;
            while (got < want && (r = fread(w->raster + got, 1, want - got, in)) > 0) got += r;
            if (got < want) memset(w->raster + got, 0, want - got);
            w->nb = nb;
            dev_post(w);
        }
        dev_worker *w = &ws[k % nDevices];
        const int rc = dev_wait(w);
        if (rc) {
            printf("Error running the 3D DCT: %s\n", dct3d_strerror(rc));
            status = 1;
            break;
        }
        uint8_t cb;
        int cbits;
        dct3d_entropy_enc_carry(ent, &cb, &cbits);
        const size_t need = (size_t)((w->bits + 7 + 7) / 8);
        if (need > joined_cap) {
            free(joined);
            joined_cap = need + need / 4;
            joined = (unsigned char *)malloc(joined_cap);
            if (!joined) {
                printf("Out of memory\n");
                status = 1;
                break;
            }
        }
        const uint64_t tb = join_carry(w->eg, w->bits, cb, cbits, joined);
        if (dct3d_entropy_enc_push_stream(ent, joined, tb, k == n_batches - 1)) {
            printf("Error in the entropy coder\n");
            status = 1;
            break;
        }
        for (int s = 0; s < w->nb; s++) printf("Frames processed: %d\n", (k * batch + s + 1) * depth);
    }
    dev_workers_destroy(ws, nDevices);  /* waits for jobs still in flight after an error */
    dct3d_entropy_enc_destroy(ent);
    free(joined);
    fclose(in);
    if (fflush(out) || fclose(out)) status = 1;
    if (!status) printf("Encoding process completed\n");
    return status;
}

/* fwrite of decoded batch k (its device's raster buffer); clears *pending; 1 on a write error */
static int write_batch(dev_worker *ws, int n, int k, int batch, int n_stacks, size_t stack_px, int depth, FILE *out,
                       int *pending) {
    const dev_worker *w = &ws[k % n];
    const int nb = (n_stacks - k * batch) < batch ? (n_stacks - k * batch) : batch;
    *pending = -1;
    if (fwrite(w->raster, 1, stack_px * nb, out) != stack_px * nb) {
        printf("Error writing the output file\n");
        return 1;
    }
    printf("Frames processed: %d\n", (k * batch + nb) * depth);
    return 0;
}

int decode_multi(const char *inName, const char *outName, int width, int height, int frames,
                 const int *platformIndices, int nDevices, int depth, int batch) {
    if (!platformIndices || nDevices <= 0) {
        printf("No device given\n");
        return 1;
    }
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
    const size_t frame = (size_t)width * height, stack_px = frame * depth;
    const int n_stacks = (frames + depth - 1) / depth;
    const int n_batches = (n_stacks + batch - 1) / batch;
    dev_worker *ws = dev_workers_create(platformIndices, nDevices, width, height, depth, stack_px * batch, 1);
    if (!ws) {
        fclose(in);
        fclose(out);
        return 1;
    }
    dct3d_entropy_dec *ent = dct3d_entropy_dec_create(width, height, depth, in, NULL, 0);
    int status = 0;
    if (!ent) {
        printf("Out of memory\n");
        status = 1;
    }
    double bits_per_value = 4.0;  /* window estimate for the first batch; then the measured rate */
    int pending = -1;             /* the decoded batch whose raster is not written yet */
    for (int k = 0; !status && k < n_batches; k++) {
        dev_worker *w = &ws[k % nDevices];
        const int s0 = k * batch, nb = (n_stacks - s0) < batch ? (n_stacks - s0) : batch;
        const double values = (double)stack_px * nb;
        size_t need = (size_t)(values * bits_per_value / 8 * 1.25) + 65536;
        int rc;
        int first = 1;
        for (;;) {
            if (dct3d_entropy_dec_window(ent, need, &w->win, &w->win_len, &w->win_bit)) {
                rc = DCT3D_EINVAL;
                break;
            }
            w->nb = nb;
            /* the previous batch's raster is written while this one decodes -- before the post when both
             * use the same (only) device's buffer */
            if (first && pending >= 0 && nDevices == 1) status = write_batch(ws, nDevices, pending, batch, n_stacks,
                                                                           stack_px, depth, out, &pending);
            dev_post(w);
            if (first && pending >= 0) status |= write_batch(ws, nDevices, pending, batch, n_stacks, stack_px, depth,
                                                            out, &pending);
            first = 0;
            rc = dev_wait(w);
            if (rc == DCT3D_ENODATA && !dct3d_entropy_dec_eof(ent) && w->win_len >= need) {
                need *= 2;  /* the batch needs more of the stream than estimated */
                continue;
            }
            if (!rc) {
                dct3d_entropy_dec_consume(ent, w->bits);
                bits_per_value = (double)(w->bits - (uint64_t)w->win_bit) / values;
            }
            break;
        }
        if (status) break;
        if (rc == DCT3D_ENODATA || rc == DCT3D_EINVAL) {
            printf("Truncated or corrupt input stream\n");
            status = 1;
            break;
        }
        if (rc) {
            printf("Error running the inverse 3D DCT: %s\n", dct3d_strerror(rc));
            status = 1;
            break;
        }
        pending = k;
    }
    if (!status && pending >= 0) status = write_batch(ws, nDevices, pending, batch, n_stacks, stack_px, depth, out,
                                                      &pending);
    dev_workers_destroy(ws, nDevices);
    dct3d_entropy_dec_destroy(ent);
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
