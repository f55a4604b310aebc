/* codec_entropy.c -- see codec_entropy.h. */
#include "codec_entropy.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "cube_utils.h"
#include "exp_golomb.h"

/* Parallel deflate (optional, dct3d_entropy_enc_set_threads): the input is cut into chunks, each chunk
 * deflated by a worker thread as raw deflate primed with the 32 KiB of input before it
 * (deflateSetDictionary) and ended with Z_SYNC_FLUSH (byte-aligned, not final; the last chunk
 * Z_FINISH); the chunks' output is concatenated in order between a zlib header (level 9) and the
 * Adler-32 of the whole input.  The result is one valid zlib stream whose INFLATED payload is the
 * reference's (the container's parity is the inflated payload); its .bin bytes differ
 * from single-stream zlib's, which stays the default. */
#define PZ_DICT 32768
typedef struct {
    unsigned char *in;   /* [dict_len bytes of dictionary][chunk bytes] */
    size_t dict_len, len;
    int last;
    unsigned char *out;
    size_t out_len;
    int done, err;
} pz_job;

typedef struct {
    int threads;
    size_t chunk;
    pthread_t *tid;
    int started;
    pthread_mutex_t mu;
    pthread_cond_t cv_work, cv_done;
    pz_job *ring;
    long ring_n, head, tail, next_work;  /* sink head, submit tail, next job to start */
    int closing;
    unsigned char *cur;  /* staging: dictionary + chunk being filled */
    size_t cur_dict, cur_len;
    uLong adler;
    int header_done;
} pz_state;

struct dct3d_entropy_enc {
    z_stream zs;
    pz_state *pz;
    FILE *out;
    unsigned char *mem;
    size_t mem_len, mem_cap;
    char *eg;
    size_t eg_cap;
    struct ExpGolombStream st;
    unsigned char zbuf[1 << 16];
    struct SlicesPositions *sp;
    int cs;
    size_t cubes;       /* cubes per stack */
    int finished;
};

static int sink(dct3d_entropy_enc *e, const unsigned char *p, size_t n) {
    if (!n) return 0;
    if (e->out) return fwrite(p, 1, n, e->out) == n ? 0 : -1;
    if (e->mem_len + n > e->mem_cap) {
        size_t cap = e->mem_cap ? e->mem_cap : 1 << 16;
        while (cap < e->mem_len + n) cap *= 2;
        unsigned char *m = (unsigned char *)realloc(e->mem, cap);
        if (!m) return -1;
        e->mem = m;
        e->mem_cap = cap;
    }
    memcpy(e->mem + e->mem_len, p, n);
    e->mem_len += n;
    return 0;
}

static void *pz_worker(void *arg) {
    pz_state *p = (pz_state *)arg;
    for (;;) {
        pthread_mutex_lock(&p->mu);
        while (p->next_work >= p->tail && !p->closing) pthread_cond_wait(&p->cv_work, &p->mu);
        if (p->next_work >= p->tail) {
            pthread_mutex_unlock(&p->mu);
            return NULL;
        }
        pz_job *j = &p->ring[p->next_work++ % p->ring_n];
        pthread_mutex_unlock(&p->mu);
        int err = 0;
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        if (deflateInit2(&zs, Z_BEST_COMPRESSION, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
            err = 1;
        } else {
            if (j->dict_len && deflateSetDictionary(&zs, j->in, (uInt)j->dict_len) != Z_OK) err = 1;
            size_t cap = deflateBound(&zs, (uLong)j->len) + 64;
            j->out = (unsigned char *)malloc(cap);
            if (!j->out) err = 1;
            zs.next_in = j->in + j->dict_len;
            zs.avail_in = (uInt)j->len;
            const int flush = j->last ? Z_FINISH : Z_SYNC_FLUSH;
            while (!err) {
                zs.next_out = j->out + j->out_len;
                zs.avail_out = (uInt)(cap - j->out_len);
                const int rc = deflate(&zs, flush);
                j->out_len = cap - zs.avail_out;
                if (rc == Z_STREAM_ERROR) err = 1;
                else if (j->last ? rc == Z_STREAM_END : (zs.avail_in == 0 && zs.avail_out != 0)) break;
                else if (rc == Z_BUF_ERROR && zs.avail_out != 0) err = 1;  /* no progress possible */
                else if (zs.avail_out == 0) {  /* grow and continue */
                    unsigned char *o = (unsigned char *)realloc(j->out, cap * 2);
                    if (!o) err = 1;
                    else { j->out = o; cap *= 2; }
                }
            }
            deflateEnd(&zs);
        }
        pthread_mutex_lock(&p->mu);
        j->err = err;
        j->done = 1;
        pthread_cond_broadcast(&p->cv_done);
        pthread_mutex_unlock(&p->mu);
    }
}

static int sink(dct3d_entropy_enc *e, const unsigned char *p, size_t n);

/* writes finished jobs in order; wait: block until the oldest job is done */
static int pz_drain(dct3d_entropy_enc *e, int wait) {
    pz_state *p = e->pz;
    int rc = 0;
    for (;;) {
        pthread_mutex_lock(&p->mu);
        if (p->head >= p->tail) {
            pthread_mutex_unlock(&p->mu);
            return rc;
        }
        pz_job *j = &p->ring[p->head % p->ring_n];
        while (!j->done && wait) pthread_cond_wait(&p->cv_done, &p->mu);
        const int ready = j->done;
        pthread_mutex_unlock(&p->mu);
        if (!ready) return rc;
        if (j->err || sink(e, j->out, j->out_len)) rc = -1;
        free(j->in);
        free(j->out);
        memset(j, 0, sizeof(*j));
        p->head++;
        wait = 0;
        if (rc) return rc;
    }
}

static int pz_submit(dct3d_entropy_enc *e, int last) {
    pz_state *p = e->pz;
    /* counted one by one, so that pz_destroy wakes and joins exactly the workers that exist */
    for (; p->started < p->threads; p->started++)
        if (pthread_create(&p->tid[p->started], NULL, pz_worker, p)) return -1;
    if (!p->header_done) {  /* zlib header: deflate, 32 KiB window, FLEVEL 3 (level 9) */
        static const unsigned char hdr[2] = {0x78, 0xDA};
        if (sink(e, hdr, 2)) return -1;
        p->header_done = 1;
    }
    while (p->tail - p->head >= p->ring_n)
        if (pz_drain(e, 1)) return -1;
    unsigned char *next = (unsigned char *)malloc(PZ_DICT + p->chunk);
    if (!next) return -1;
    /* the next chunk's dictionary: the last 32 KiB of all input so far */
    const size_t have = p->cur_len;  /* dictionary + chunk bytes in cur */
    const size_t nd = have < PZ_DICT ? have : PZ_DICT;
    memcpy(next, p->cur + have - nd, nd);
    pthread_mutex_lock(&p->mu);
    pz_job *j = &p->ring[p->tail % p->ring_n];
    j->in = p->cur;
    j->dict_len = p->cur_dict;
    j->len = p->cur_len - p->cur_dict;
    j->last = last;
    j->out = NULL;
    j->out_len = 0;
    j->done = j->err = 0;
    p->tail++;
    pthread_cond_signal(&p->cv_work);
    pthread_mutex_unlock(&p->mu);
    p->cur = next;
    p->cur_dict = p->cur_len = nd;
    return pz_drain(e, 0);
}

static int pz_feed(dct3d_entropy_enc *e, const unsigned char *in, size_t n) {
    pz_state *p = e->pz;
    while (n) {
        size_t room = p->cur_dict + p->chunk - p->cur_len;
        size_t take = n < room ? n : room;
        memcpy(p->cur + p->cur_len, in, take);
        p->adler = adler32(p->adler, in, (uInt)take);
        p->cur_len += take;
        in += take;
        n -= take;
        if (p->cur_len == p->cur_dict + p->chunk && pz_submit(e, 0)) return -1;
    }
    return 0;
}

static int pz_finish(dct3d_entropy_enc *e) {
    pz_state *p = e->pz;
    if (pz_submit(e, 1)) return -1;
    while (p->head < p->tail)
        if (pz_drain(e, 1)) return -1;
    const unsigned char tr[4] = {(unsigned char)(p->adler >> 24), (unsigned char)(p->adler >> 16),
                                 (unsigned char)(p->adler >> 8), (unsigned char)p->adler};
    return sink(e, tr, 4);
}

static void pz_destroy(pz_state *p) {
    if (!p) return;
    pthread_mutex_lock(&p->mu);
    p->closing = 1;
    pthread_cond_broadcast(&p->cv_work);
    pthread_mutex_unlock(&p->mu);
    for (int t = 0; t < p->started; t++) pthread_join(p->tid[t], NULL);
    for (long i = p->head; i < p->tail; i++) {
        free(p->ring[i % p->ring_n].in);
        free(p->ring[i % p->ring_n].out);
    }
    pthread_mutex_destroy(&p->mu);
    pthread_cond_destroy(&p->cv_work);
    pthread_cond_destroy(&p->cv_done);
    free(p->ring);
    free(p->tid);
    free(p->cur);
    free(p);
}

int dct3d_entropy_enc_set_threads(dct3d_entropy_enc *e, int threads, size_t chunk_bytes) {
    if (!e || e->pz || e->finished || e->zs.total_in) return -1;
    if (threads <= 1) return 0;  /* the single zlib stream (the reference's bytes) */
    pz_state *p = (pz_state *)calloc(1, sizeof(*p));
    if (!p) return -1;
    p->threads = threads;
    p->chunk = chunk_bytes ? chunk_bytes : (size_t)256 << 10;
    p->ring_n = 2 * threads;
    p->tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    p->ring = (pz_job *)calloc((size_t)p->ring_n, sizeof(pz_job));
    p->cur = (unsigned char *)malloc(PZ_DICT + p->chunk);
    p->adler = adler32(0L, Z_NULL, 0);
    pthread_mutex_init(&p->mu, NULL);
    pthread_cond_init(&p->cv_work, NULL);
    pthread_cond_init(&p->cv_done, NULL);
    e->pz = p;
    if (!p->tid || !p->ring || !p->cur) {
        pz_destroy(p);
        e->pz = NULL;
        return -1;
    }
    return 0;
}

static int deflate_all(dct3d_entropy_enc *e, const unsigned char *in, size_t n, int flush) {
    if (e->pz) {
        if (pz_feed(e, in, n)) return -1;
        return flush == Z_FINISH ? pz_finish(e) : 0;
    }
    e->zs.next_in = (Bytef *)in;
    e->zs.avail_in = (uInt)n;
    for (;;) {
        e->zs.next_out = e->zbuf;
        e->zs.avail_out = sizeof(e->zbuf);
        int rc = deflate(&e->zs, flush);
        if (rc == Z_STREAM_ERROR) return -1;
        if (sink(e, e->zbuf, sizeof(e->zbuf) - e->zs.avail_out)) return -1;
        if (flush == Z_FINISH) {
            if (rc == Z_STREAM_END) return 0;
        } else if (e->zs.avail_in == 0 && e->zs.avail_out != 0) {
            return 0;
        }
    }
}

dct3d_entropy_enc *dct3d_entropy_enc_create(int width, int height, int depth, FILE *out) {
    if (width <= 0 || height <= 0 || width % 8 || height % 8 || (depth != 8 && depth != 4)) return NULL;
    dct3d_entropy_enc *e = (dct3d_entropy_enc *)calloc(1, sizeof(*e));
    if (!e) return NULL;
    e->out = out;
    e->cs = 64 * depth;
    e->cubes = (size_t)(width / 8) * (height / 8);
    e->sp = cubeUtils_diagonalSlices(8, 8, depth);
    /* worst case: 63 bits per value (|v| < 2^31) -> 8 bytes per value */
    e->eg_cap = e->cubes * e->cs * 8 + 16;
    e->eg = (char *)calloc(e->eg_cap, 1);
    if (!e->sp || !e->eg || deflateInit(&e->zs, Z_BEST_COMPRESSION) != Z_OK) {  /* encoder.c:136-139 */
        cubeUtils_deallocatePositions(e->sp);
        free(e->eg);
        free(e);
        return NULL;
    }
    e->st.buffer = e->eg;
    e->st.bitPosition = 8;
    e->st.bufferPosition = 0;
    return e;
}

int dct3d_entropy_enc_push(dct3d_entropy_enc *e, const int32_t *q, int is_last) {
    if (e->finished) return -1;
    /* applyExpGolombCoding (encoder.c:60-71): diagonal order inside each cube */
    for (size_t c = 0; c < e->cubes; c++) {
        const int32_t *cube = q + c * e->cs;
        for (int i = 0; i < e->sp->length; i++) {
            const struct ThreeDimensionalCoordinates p = e->sp->positions[i];
            expGolomb_writeValue(&e->st, cube[p.x + p.y * 8 + p.z * 64]);
        }
    }
    const int size = e->st.bufferPosition;
    if (!is_last) {
        if (deflate_all(e, (const unsigned char *)e->eg, (size_t)size, Z_NO_FLUSH)) return -1;
        expGolomb_freeBuffer(&e->st, size, 1);  /* keep the partial byte (encoder.c:268) */
        return 0;
    }
    e->finished = 1;
    return deflate_all(e, (const unsigned char *)e->eg, (size_t)size + 1, Z_FINISH);  /* encoder.c:270 */
}

void dct3d_entropy_enc_carry(const dct3d_entropy_enc *e, uint8_t *byte, int *bits) {
    /* after expGolomb_freeBuffer the partial byte sits at position 0 */
    *bits = 8 - e->st.bitPosition;
    *byte = *bits ? (uint8_t)e->eg[e->st.bufferPosition] : 0;
}

int dct3d_entropy_enc_push_stream(dct3d_entropy_enc *e, const unsigned char *bytes, uint64_t total_bits, int is_last) {
    if (e->finished || e->st.bufferPosition != 0) return -1;
    const size_t complete = (size_t)(total_bits / 8);
    const int rem = (int)(total_bits % 8);
    if (is_last) {
        e->finished = 1;
        if (rem) return deflate_all(e, bytes, complete + 1, Z_FINISH);
        /* the reference deflates bufferPosition + 1 bytes: a whole-byte stream ends with one zero byte */
        if (complete && deflate_all(e, bytes, complete, Z_NO_FLUSH)) return -1;
        static const unsigned char zero = 0;
        return deflate_all(e, &zero, 1, Z_FINISH);
    }
    if (deflate_all(e, bytes, complete, Z_NO_FLUSH)) return -1;
    e->eg[0] = rem ? (char)bytes[complete] : 0;
    e->st.bitPosition = 8 - rem;
    e->st.bufferPosition = 0;
    return 0;
}

const unsigned char *dct3d_entropy_enc_memory(const dct3d_entropy_enc *e, size_t *len) {
    if (len) *len = e->mem_len;
    return e->mem;
}

void dct3d_entropy_enc_destroy(dct3d_entropy_enc *e) {
    if (!e) return;
    pz_destroy(e->pz);
    deflateEnd(&e->zs);
    cubeUtils_deallocatePositions(e->sp);
    free(e->eg);
    free(e->mem);
    free(e);
}

/* ------------------------------------------------------------------------------------------ */
struct dct3d_entropy_dec {
    z_stream zs;
    FILE *in;
    const unsigned char *mem;
    size_t mem_len, mem_pos;
    int zeof, ieof;
    unsigned char *buf;   /* inflated, unconsumed bytes */
    size_t len, cap;
    struct ExpGolombStream st;
    unsigned char ibuf[1 << 16];
    struct SlicesPositions *sp;
    int cs;
    size_t cubes;
};

dct3d_entropy_dec *dct3d_entropy_dec_create(int width, int height, int depth, FILE *in, const unsigned char *mem,
                                            size_t len) {
    if (width <= 0 || height <= 0 || width % 8 || height % 8 || (depth != 8 && depth != 4)) return NULL;
    dct3d_entropy_dec *d = (dct3d_entropy_dec *)calloc(1, sizeof(*d));
    if (!d) return NULL;
    d->in = in;
    d->mem = mem;
    d->mem_len = len;
    d->cs = 64 * depth;
    d->cubes = (size_t)(width / 8) * (height / 8);
    d->sp = cubeUtils_diagonalSlices(8, 8, depth);
    d->cap = 1 << 20;
    d->buf = (unsigned char *)malloc(d->cap);
    if (!d->sp || !d->buf || inflateInit(&d->zs) != Z_OK) {
        cubeUtils_deallocatePositions(d->sp);
        free(d->buf);
        free(d);
        return NULL;
    }
    d->st.buffer = (char *)d->buf;
    d->st.bitPosition = 8;
    d->st.bufferPosition = 0;
    return d;
}

/* make at least `need` unconsumed bytes available (or hit the end of the stream) */
static int refill(dct3d_entropy_dec *d, size_t need) {
    for (;;) {
        const size_t avail = d->len - (size_t)d->st.bufferPosition;
        if (avail >= need || d->zeof) return 0;
        /* compact: drop consumed bytes (decoder.c:233-235) */
        if (d->st.bufferPosition > 0) {
            memmove(d->buf, d->buf + d->st.bufferPosition, avail);
            d->len = avail;
            d->st.bufferPosition = 0;
        }
        if (d->cap - d->len < (1 << 16)) {
            unsigned char *b = (unsigned char *)realloc(d->buf, d->cap * 2);
            if (!b) return -1;
            d->buf = b;
            d->cap *= 2;
            d->st.buffer = (char *)b;
        }
        if (d->zs.avail_in == 0 && !d->ieof) {
            if (d->in) {
                size_t r = fread(d->ibuf, 1, sizeof(d->ibuf), d->in);
                if (r == 0) d->ieof = 1;
                d->zs.next_in = d->ibuf;
                d->zs.avail_in = (uInt)r;
            } else {
                size_t r = d->mem_len - d->mem_pos;
                if (r > (1u << 30)) r = 1u << 30;
                if (r == 0) d->ieof = 1;
                d->zs.next_in = (Bytef *)(d->mem + d->mem_pos);
                d->zs.avail_in = (uInt)r;
                d->mem_pos += r;
            }
        }
        d->zs.next_out = d->buf + d->len;
        d->zs.avail_out = (uInt)(d->cap - d->len);
        const int rc = inflate(&d->zs, Z_NO_FLUSH);
        d->len = d->cap - d->zs.avail_out;
        if (rc == Z_STREAM_END) d->zeof = 1;
        else if (rc != Z_OK && rc != Z_BUF_ERROR) return -1;
        else if (rc == Z_BUF_ERROR && d->ieof) d->zeof = 1;  /* truncated input */
    }
}

int dct3d_entropy_dec_window(dct3d_entropy_dec *d, size_t need, const unsigned char **p, size_t *len, int *bit) {
    if (refill(d, need)) return -1;
    *p = d->buf + d->st.bufferPosition;
    *len = d->len - (size_t)d->st.bufferPosition;
    *bit = 8 - d->st.bitPosition;
    return 0;
}

void dct3d_entropy_dec_consume(dct3d_entropy_dec *d, uint64_t bits) {
    d->st.bufferPosition += (int)(bits / 8);
    d->st.bitPosition = 8 - (int)(bits % 8);
}

int dct3d_entropy_dec_eof(const dct3d_entropy_dec *d) { return d->zeof; }

int dct3d_entropy_dec_pull(dct3d_entropy_dec *d, int32_t *q) {
    for (size_t c = 0; c < d->cubes; c++) {
        int32_t *cube = q + c * d->cs;
        for (int i = 0; i < d->sp->length; i++) {
            if (refill(d, 16)) return -1;
            /* a codeword needs at most 8 bytes; past the end the stream is corrupt */
            if (d->len - (size_t)d->st.bufferPosition < 9) {
                if (d->len - (size_t)d->st.bufferPosition == 0) return -1;
                memset(d->buf + d->len, 0xFF, 16 < d->cap - d->len ? 16 : d->cap - d->len);
            }
            const struct ThreeDimensionalCoordinates p = d->sp->positions[i];
            cube[p.x + p.y * 8 + p.z * 64] = expGolomb_readValue(&d->st);
            if ((size_t)d->st.bufferPosition > d->len) return -1;
        }
    }
    return 0;
}

void dct3d_entropy_dec_destroy(dct3d_entropy_dec *d) {
    if (!d) return;
    inflateEnd(&d->zs);
    cubeUtils_deallocatePositions(d->sp);
    free(d->buf);
    free(d);
}

int dct3d_codec_entropy_encode(const int32_t *q, int width, int height, int n_stacks, int depth, unsigned char **out,
                               size_t *out_len) {
    return dct3d_codec_entropy_encode_mt(q, width, height, n_stacks, depth, 1, 0, out, out_len);
}

int dct3d_codec_entropy_encode_mt(const int32_t *q, int width, int height, int n_stacks, int depth, int threads,
                                  size_t chunk_bytes, unsigned char **out, size_t *out_len) {
    if (!out || !out_len || n_stacks <= 0) return -1;
    dct3d_entropy_enc *e = dct3d_entropy_enc_create(width, height, depth, NULL);
    if (!e) return -1;
    if (dct3d_entropy_enc_set_threads(e, threads, chunk_bytes)) {
        dct3d_entropy_enc_destroy(e);
        return -1;
    }
    const size_t per = e->cubes * (size_t)e->cs;
    for (int s = 0; s < n_stacks; s++)
        if (dct3d_entropy_enc_push(e, q + per * s, s == n_stacks - 1)) {
            dct3d_entropy_enc_destroy(e);
            return -1;
        }
    *out_len = e->mem_len;
    *out = e->mem;
    e->mem = NULL;
    dct3d_entropy_enc_destroy(e);
    return 0;
}

int dct3d_codec_entropy_decode(const unsigned char *bin, size_t len, int width, int height, int n_stacks, int depth,
                               int32_t *q) {
    dct3d_entropy_dec *d = dct3d_entropy_dec_create(width, height, depth, NULL, bin, len);
    if (!d) return -1;
    const size_t per = d->cubes * (size_t)d->cs;
    int rc = 0;
    for (int s = 0; s < n_stacks && !rc; s++) rc = dct3d_entropy_dec_pull(d, q + per * s);
    dct3d_entropy_dec_destroy(d);
    return rc;
}

void dct3d_codec_free(void *p) { free(p); }
