/*
 * oracle/java_dct3d.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * A plain-C restatement of the reference's *Java* codec semantics for the hot path
 * (the parity target named in BASELINE.json north_star).  Only tests/, the
 * __graft_entry__.smoke() checker and bench.py's cpu_baseline leg may load this.
 *
 * What it restates (file:line under /root/reference/3d-DCT-video-encoding/src/br/jpiccoli/video/):
 *   - Transform constants            dct/Transform.java:20-21
 *   - DCT.initialize coefficient     dct/DCT.java:77-140  (grouping by (long)(c*1e9) in a
 *     grouping + Java 8 HashMap        java.util.HashMap<Long,..>; fold order = HashMap
 *     iteration order                  iteration order, emulated exactly below)
 *   - DCT.createSums memoisation     dct/DCT.java:155-163, dct/Sum.java:41-52
 *   - DCT.apply fold                 dct/DCT.java:41-59   (output += sum * coefficient)
 *   - Transform.run thread pool      dct/Transform.java:63-104 (one task per cube)
 *   - Encoder quantisation           Encoder.java:75-89   (Math.round, cube-major repack)
 *   - Decoder dequantisation         Decoder.java:78-96
 *   - InverseDCT.initialize/apply    dct/InverseDCT.java:33-133 (skip |x|<=1e-9, clamp)
 *   - (byte) truncation on write     Decoder.java:107-117
 *   - CubeUtils.diagonalSlices       CubeUtils.java:7-41
 *   - ExpGolombWriter/Reader         ExpGolombWriter.java:19-49, ExpGolombReader.java:19-63
 *
 * Parity pinning: there is no JDK in this image and the reference ships no tests or golden
 * vectors.  This restatement is pinned (tests/test_oracle.py) by
 *   (1) the reference's own C host helpers (CubeUtils.c, ExpGolomb.c, readCubes/writeCubes,
 *       applyQuantization/applyDequantization) compiled from /root/reference into oracle/_ref,
 *   (2) the structural counts of the Java grouping (11,567 multiplications / 2,319 distinct
 *       sums per 8^3 cube; 4,301 per 8x8x4),
 *   (3) an independent arbitrary-precision evaluation of the DCT formula (quantised ints must
 *       agree wherever the exact value is not within 1e-9 of a rounding tie).
 * Residual unpinned item: Math.cos differs from the correctly rounded value.  glibc cos() is used
 * and is correctly rounded at every argument the plan evaluates; every group key except those of
 * the exactly rational coefficients (+-1/32, +-1/16) is stable under any 1-ulp cosine error
 * (tests/test_plan.py::test_libm_cos_correctly_rounded_at_plan_arguments,
 * ::test_grouping_keys_stable_under_cos_ulp).
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off; no FMA contraction, like javac/HotSpot).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* Java primitives                                                                              */
/* ------------------------------------------------------------------------------------------ */

/* (long) d : JLS 5.1.3 narrowing, truncation toward zero, saturating, NaN -> 0. */
static int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

/* Math.round(double) (Java 8): round half up, computed exactly (no floor(x+0.5) rounding). */
int64_t oracle_java_round(double a) {
    if (a != a) return 0;
    double f = floor(a);
    double r = a - f; /* exact for |a| < 2^52 */
    int64_t n = java_d2l(f);
    return (r >= 0.5) ? n + 1 : n;
}

/* ------------------------------------------------------------------------------------------ */
/* java.util.HashMap<Long, V> (Java 8) insertion/iteration-order emulation                     */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    uint32_t hash;
    int64_t key;
    int val;
    int next;
} jnode;

typedef struct {
    int *tab;
    int cap, size, thr;
    jnode *nodes;
    int nn, ncap;
    int treeified; /* set if Java would have treeified a bin (iteration order then differs) */
} jmap;

static uint32_t jmap_hash(int64_t key) {
    uint64_t v = (uint64_t)key;
    uint32_t h = (uint32_t)(v ^ (v >> 32)); /* Long.hashCode */
    return h ^ (h >> 16);                   /* HashMap.hash spread */
}

static void jmap_resize(jmap *m) {
    if (m->cap == 0) {
        m->cap = 16;
        m->thr = 12;
        m->tab = (int *)malloc(sizeof(int) * 16);
        for (int i = 0; i < 16; i++) m->tab[i] = -1;
        return;
    }
    int oc = m->cap, nc = oc * 2;
    int *nt = (int *)malloc(sizeof(int) * nc);
    for (int j = 0; j < oc; j++) {
        int loH = -1, loT = -1, hiH = -1, hiT = -1;
        for (int e = m->tab[j]; e >= 0;) {
            int nx = m->nodes[e].next;
            m->nodes[e].next = -1;
            if ((m->nodes[e].hash & (uint32_t)oc) == 0) {
                if (loT < 0) loH = e; else m->nodes[loT].next = e;
                loT = e;
            } else {
                if (hiT < 0) hiH = e; else m->nodes[hiT].next = e;
                hiT = e;
            }
            e = nx;
        }
        nt[j] = loH;
        nt[j + oc] = hiH;
    }
    free(m->tab);
    m->tab = nt;
    m->cap = nc;
    m->thr = m->thr * 2;
}

static int jmap_get(const jmap *m, int64_t key) {
    if (m->cap == 0) return -1;
    uint32_t h = jmap_hash(key);
    for (int e = m->tab[h & (uint32_t)(m->cap - 1)]; e >= 0; e = m->nodes[e].next)
        if (m->nodes[e].key == key) return m->nodes[e].val;
    return -1;
}

/* putVal for a key known to be absent (DCT.java:85-91 does get() then put()). */
static void jmap_put_new(jmap *m, int64_t key, int val) {
    if (m->cap == 0) jmap_resize(m);
    if (m->nn == m->ncap) {
        m->ncap = m->ncap ? m->ncap * 2 : 64;
        m->nodes = (jnode *)realloc(m->nodes, sizeof(jnode) * m->ncap);
    }
    int id = m->nn++;
    uint32_t h = jmap_hash(key);
    m->nodes[id].hash = h;
    m->nodes[id].key = key;
    m->nodes[id].val = val;
    m->nodes[id].next = -1;
    int idx = (int)(h & (uint32_t)(m->cap - 1));
    if (m->tab[idx] < 0) {
        m->tab[idx] = id;
    } else {
        int p = m->tab[idx], binCount = 0;
        while (m->nodes[p].next >= 0) { p = m->nodes[p].next; binCount++; }
        m->nodes[p].next = id;
        if (binCount >= 7) {                /* TREEIFY_THRESHOLD - 1 */
            if (m->cap < 64) jmap_resize(m); /* MIN_TREEIFY_CAPACITY */
            else m->treeified = 1;
        }
    }
    if (++m->size > m->thr) jmap_resize(m);
}

static void jmap_free(jmap *m) {
    free(m->tab);
    free(m->nodes);
    memset(m, 0, sizeof(*m));
}

/* ------------------------------------------------------------------------------------------ */
/* Plan: DCT.initialize + createSums, InverseDCT.initialize                                    */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    double coef;
    int sum_id;    /* memoised Sum index (DCT.createSums) */
} jmult;

typedef struct {
    int cw, ch, cd, cs;
    /* forward: per output coefficient k (cube-local z*ch*cw + y*cw + x), the multiplication list
       in HashMap iteration order (DCT.java:98: new LinkedList<>(map.values())). */
    int *mult_off;      /* [cs+1] offsets into mults */
    jmult *mults;
    int n_mults;
    /* distinct sums (DCT.java:155-163): member lists of cube-local input indices */
    int n_sums;
    int *sum_off;       /* [n_sums+1] */
    int *sum_members;   /* cube-local n = z*ch*cw + y*cw + x */
    /* per (k, group) member map for convenience: group_of[k*cs + n] = group index in fold order */
    int16_t *group_of;
    /* inverse: InverseDCT.coefficients[n][k] */
    double *inv_coef;   /* [cs*cs] */
    int treeified;
} jplan;

/* Residual study only (tools/cos_ulp_sensitivity.py, tests/test_cos_residual.py): an alternative
 * plan whose Math.cos differs from glibc's correctly rounded cos at chosen arguments by +-1 ulp, and/or
 * whose exactly rational coefficients (c * 1E9 within 1e-6 of an integer K, DCT.java:112-116) take the
 * other integer key.  key_flip: 0 none, 1 toggle (K <-> K - sign), 2 all to K - sign, 3 all to K.
 * The default plan (oracle_plan_create) uses none of this. */
typedef struct {
    const double *args;
    const int8_t *delta;
    int n;
    int key_flip;
} cosalt;

static double java_cos(double a, const cosalt *alt) {
    double c = cos(a);
    if (alt)
        for (int i = 0; i < alt->n; i++)
            if (alt->args[i] == a && alt->delta[i]) {
                c = nextafter(c, alt->delta[i] > 0 ? INFINITY : -INFINITY);
                break;
            }
    return c;
}

static int64_t java_key(double coef, const cosalt *alt) {
    int64_t key = java_d2l(coef * 1E9);
    if (!alt || !alt->key_flip) return key;
    const double x = coef * 1E9, K = nearbyint(x);
    if (fabs(x - K) >= 1e-6 || K == 0.0) return key;   /* not a rational coefficient's key */
    const int64_t ki = (int64_t)K, lo = ki - (x > 0 ? 1 : -1); /* the two candidate keys */
    switch (alt->key_flip) {
    case 1: return key == ki ? lo : ki;
    case 2: return lo;
    default: return ki;
    }
}

static double java_coef_alt(const jplan *p, double scale, int k0, int k1, int k2, int n0, int n1, int n2,
                            const cosalt *alt) {
    /* Transform.java:20-21 */
    const double INVERSE_SQRT_2 = 1.0 / sqrt(2.0);
    /* DCT.java:81-84: Math.PI / (float) N -> double */
    const double piOverWidth = M_PI / (double)(float)p->cw;
    const double piOverHeight = M_PI / (double)(float)p->ch;
    const double piOverDepth = M_PI / (double)(float)p->cd;
    double c0 = k0 == 0 ? INVERSE_SQRT_2 : 1.0;
    double c1 = k1 == 0 ? INVERSE_SQRT_2 : 1.0;
    double c2 = k2 == 0 ? INVERSE_SQRT_2 : 1.0;
    /* (n + 0.5f) is a float; evaluation strictly left to right (DCT.java:110) */
    double a0 = piOverDepth * (double)((float)n0 + 0.5f) * (double)k0;
    double a1 = piOverHeight * (double)((float)n1 + 0.5f) * (double)k1;
    double a2 = piOverWidth * (double)((float)n2 + 0.5f) * (double)k2;
    double c = scale * c0;
    c = c * c1;
    c = c * c2;
    c = c * java_cos(a0, alt);
    c = c * java_cos(a1, alt);
    c = c * java_cos(a2, alt);
    return c;
}

/* simple open-addressing set of member lists for createSums memoisation */
typedef struct { uint64_t h; int id; } sumslot;

static uint64_t hash_members(const int *m, int n) {
    /* order-independent (Java Set equality): sort-free XOR/sum mix over a sorted copy */
    uint64_t a = 1469598103934665603ULL;
    for (int i = 0; i < n; i++) {
        uint64_t x = (uint64_t)m[i] * 0x9E3779B97F4A7C15ULL;
        x ^= x >> 29;
        a += x * 0xBF58476D1CE4E5B9ULL;
    }
    return a ^ (uint64_t)n;
}

static int cmp_int(const void *a, const void *b) {
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

static jplan *plan_create(int cw, int ch, int cd, const cosalt *alt) {
    jplan *p = (jplan *)calloc(1, sizeof(jplan));
    p->cw = cw; p->ch = ch; p->cd = cd;
    int cs = cw * ch * cd;
    p->cs = cs;
    /* Transform.java:20: DIMENSIONAL_FACTOR = sqrt(pow(2.0f, 3.0f)); DCT.java:79 */
    const double DIMENSIONAL_FACTOR = sqrt(pow(2.0, 3.0));
    const double scale = DIMENSIONAL_FACTOR / sqrt((double)cs);

    p->mult_off = (int *)malloc(sizeof(int) * (cs + 1));
    int mcap = cs * 64;
    p->mults = (jmult *)malloc(sizeof(jmult) * mcap);
    p->group_of = (int16_t *)malloc(sizeof(int16_t) * (size_t)cs * cs);
    /* temporary member storage per group */
    int *gcount = (int *)malloc(sizeof(int) * cs);
    int *gmem = (int *)malloc(sizeof(int) * (size_t)cs * cs);
    int *gfirst_coef_idx = (int *)malloc(sizeof(int) * cs);
    double *gcoef = (double *)malloc(sizeof(double) * cs);

    /* sums memo table */
    int scap = 1 << 16;
    sumslot *slots = (sumslot *)malloc(sizeof(sumslot) * scap);
    for (int i = 0; i < scap; i++) slots[i].id = -1;
    int sum_mem_cap = cs * 1024;
    p->sum_off = (int *)malloc(sizeof(int) * (scap + 1));
    p->sum_members = (int *)malloc(sizeof(int) * sum_mem_cap);
    p->sum_off[0] = 0;
    p->n_sums = 0;
    int *tmp = (int *)malloc(sizeof(int) * cs);

    p->n_mults = 0;
    int k = 0;
    for (int k0 = 0; k0 < cd; k0++)
        for (int k1 = 0; k1 < ch; k1++)
            for (int k2 = 0; k2 < cw; k2++, k++) {
                jmap m;
                memset(&m, 0, sizeof(m));
                int ng = 0;
                for (int i = 0; i < cs; i++) p->group_of[(size_t)k * cs + i] = -1;
                for (int n0 = 0; n0 < cd; n0++)
                    for (int n1 = 0; n1 < ch; n1++)
                        for (int n2 = 0; n2 < cw; n2++) {
                            double coef = java_coef_alt(p, scale, k0, k1, k2, n0, n1, n2, alt);
                            int64_t key = java_key(coef, alt);
                            if (key == 0) continue; /* DCT.java:84 */
                            int g = jmap_get(&m, key);
                            if (g < 0) {
                                g = ng++;
                                gcount[g] = 0;
                                gcoef[g] = coef; /* first inserted keeps its coefficient */
                                jmap_put_new(&m, key, g);
                            }
                            gmem[(size_t)g * cs + gcount[g]++] = (n0 * ch + n1) * cw + n2;
                        }
                if (m.treeified) p->treeified = 1;
                /* iterate values() in table order -> fold order */
                p->mult_off[k] = p->n_mults;
                int order = 0;
                for (int b = 0; b < m.cap; b++)
                    for (int e = m.tab[b]; e >= 0; e = m.nodes[e].next) {
                        int g = m.nodes[e].val;
                        if (p->n_mults == mcap) {
                            mcap *= 2;
                            p->mults = (jmult *)realloc(p->mults, sizeof(jmult) * mcap);
                        }
                        /* createSums: memoise identical member sets across all k */
                        int cnt = gcount[g];
                        memcpy(tmp, gmem + (size_t)g * cs, sizeof(int) * cnt);
                        qsort(tmp, cnt, sizeof(int), cmp_int);
                        uint64_t hh = hash_members(tmp, cnt);
                        int slot = (int)(hh & (uint64_t)(scap - 1)), sid = -1;
                        while (slots[slot].id >= 0) {
                            if (slots[slot].h == hh) {
                                int id = slots[slot].id;
                                int len = p->sum_off[id + 1] - p->sum_off[id];
                                if (len == cnt && !memcmp(p->sum_members + p->sum_off[id], tmp, sizeof(int) * cnt)) {
                                    sid = id;
                                    break;
                                }
                            }
                            slot = (slot + 1) & (scap - 1);
                        }
                        if (sid < 0) {
                            sid = p->n_sums++;
                            slots[slot].h = hh;
                            slots[slot].id = sid;
                            int base = p->sum_off[sid];
                            if (base + cnt > sum_mem_cap) {
                                sum_mem_cap = 2 * (base + cnt);
                                p->sum_members = (int *)realloc(p->sum_members, sizeof(int) * sum_mem_cap);
                            }
                            memcpy(p->sum_members + base, tmp, sizeof(int) * cnt);
                            p->sum_off[sid + 1] = base + cnt;
                        }
                        p->mults[p->n_mults].coef = gcoef[g];
                        p->mults[p->n_mults].sum_id = sid;
                        p->n_mults++;
                        for (int i = 0; i < cnt; i++) p->group_of[(size_t)k * cs + gmem[(size_t)g * cs + i]] = (int16_t)order;
                        order++;
                    }
                jmap_free(&m);
            }
    p->mult_off[cs] = p->n_mults;

    /* InverseDCT.initialize (InverseDCT.java:87-133) */
    p->inv_coef = (double *)malloc(sizeof(double) * (size_t)cs * cs);
    for (int n0 = 0; n0 < cd; n0++)
        for (int n1 = 0; n1 < ch; n1++)
            for (int n2 = 0; n2 < cw; n2++) {
                int on = (n0 * ch + n1) * cw + n2;
                for (int k0 = 0; k0 < cd; k0++)
                    for (int k1 = 0; k1 < ch; k1++)
                        for (int k2 = 0; k2 < cw; k2++) {
                            int ik = (k0 * ch + k1) * cw + k2;
                            p->inv_coef[(size_t)on * cs + ik] = java_coef_alt(p, scale, k0, k1, k2, n0, n1, n2, alt);
                        }
            }
    free(gcount); free(gmem); free(gfirst_coef_idx); free(gcoef); free(slots); free(tmp);
    return p;
}

jplan *oracle_plan_create(int cw, int ch, int cd) { return plan_create(cw, ch, cd, NULL); }

/* the residual study's alternative plan (cosalt above): n (argument, +-1 ulp) pairs, key_flip mode */
jplan *oracle_plan_create_alt(int cw, int ch, int cd, const double *args, const int8_t *delta, int n, int key_flip) {
    const cosalt alt = {args, delta, n, key_flip};
    return plan_create(cw, ch, cd, &alt);
}

void oracle_plan_destroy(jplan *p) {
    if (!p) return;
    free(p->mult_off); free(p->mults); free(p->sum_off); free(p->sum_members);
    free(p->group_of); free(p->inv_coef); free(p);
}

int oracle_plan_n_mults(const jplan *p) { return p->n_mults; }
int oracle_plan_n_sums(const jplan *p) { return p->n_sums; }
int oracle_plan_treeified(const jplan *p) { return p->treeified; }
int oracle_plan_n_groups(const jplan *p, int k) { return p->mult_off[k + 1] - p->mult_off[k]; }
double oracle_plan_group_coef(const jplan *p, int k, int g) { return p->mults[p->mult_off[k] + g].coef; }
/* group_of[n] for coefficient k (fold order index), -1 if the input was dropped (key == 0) */
void oracle_plan_group_of(const jplan *p, int k, int16_t *out) {
    memcpy(out, p->group_of + (size_t)k * p->cs, sizeof(int16_t) * p->cs);
}
double oracle_plan_inv_coef(const jplan *p, int n, int k) { return p->inv_coef[(size_t)n * p->cs + k]; }

/* ------------------------------------------------------------------------------------------ */
/* Transform.run: one task per cube on a fixed pool (Transform.java:74-104)                    */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    const jplan *p;
    const void *in;
    double *out;
    int W, H, F;
    int n_cubes;
    int next;
    pthread_mutex_t mu;
    int kind; /* 0 forward (u8 in), 1 inverse (double in) */
} jpool;

/* DCT.apply (DCT.java:41-59): output[k] += sum(members) * coefficient, sums memoised per cube */
static void dct_apply(const jplan *p, const uint8_t *in, double *out, int W, int H, int x, int y, int z,
                      double *cache, unsigned char *have) {
    const int frameSize = W * H;
    const int offset = z * frameSize + y * W + x;
    memset(have, 0, (size_t)p->n_sums);
    int k = 0;
    for (int k0 = 0; k0 < p->cd; k0++)
        for (int k1 = 0; k1 < p->ch; k1++)
            for (int k2 = 0; k2 < p->cw; k2++, k++) {
                size_t o = (size_t)offset + (size_t)k0 * frameSize + (size_t)k1 * W + k2;
                double acc = out[o];
                for (int mi = p->mult_off[k]; mi < p->mult_off[k + 1]; mi++) {
                    int sid = p->mults[mi].sum_id;
                    double s;
                    if (have[sid]) {
                        s = cache[sid];
                    } else {
                        s = 0.0;
                        for (int t = p->sum_off[sid]; t < p->sum_off[sid + 1]; t++) {
                            int n = p->sum_members[t];
                            int n2 = n % p->cw, n1 = (n / p->cw) % p->ch, n0 = n / (p->cw * p->ch);
                            s += (double)in[offset + n0 * frameSize + n1 * W + n2];
                        }
                        cache[sid] = s;
                        have[sid] = 1;
                    }
                    double prod = s * p->mults[mi].coef;
                    acc = acc + prod;
                }
                out[o] = acc;
            }
}

/* InverseDCT.apply (InverseDCT.java:33-82) */
static void idct_apply(const jplan *p, const double *in, double *out, int W, int H, int x, int y, int z,
                       double *nzv, int *nzi) {
    const int frameSize = W * H;
    const int offset = z * frameSize + y * W + x;
    int nnz = 0;
    for (int k0 = 0; k0 < p->cd; k0++)
        for (int k1 = 0; k1 < p->ch; k1++)
            for (int k2 = 0; k2 < p->cw; k2++) {
                double v = in[offset + k0 * frameSize + k1 * W + k2];
                if (fabs(v) > 1E-9) {
                    nzv[nnz] = v;
                    nzi[nnz++] = (k0 * p->ch + k1) * p->cw + k2;
                }
            }
    for (int n0 = 0; n0 < p->cd; n0++)
        for (int n1 = 0; n1 < p->ch; n1++)
            for (int n2 = 0; n2 < p->cw; n2++) {
                int on = (n0 * p->ch + n1) * p->cw + n2;
                size_t o = (size_t)offset + (size_t)n0 * frameSize + (size_t)n1 * W + n2;
                double acc = out[o];
                const double *row = p->inv_coef + (size_t)on * p->cs;
                for (int i = 0; i < nnz; i++) {
                    double prod = nzv[i] * row[nzi[i]];
                    acc = acc + prod;
                }
                out[o] = acc;
            }
    for (int n0 = 0; n0 < p->cd; n0++)
        for (int n1 = 0; n1 < p->ch; n1++)
            for (int n2 = 0; n2 < p->cw; n2++) {
                size_t o = (size_t)offset + (size_t)n0 * frameSize + (size_t)n1 * W + n2;
                double v = out[o];
                double mn = (255.0 < v) ? 255.0 : v; /* Math.min(255.0d, v) */
                out[o] = (0.0 > mn) ? 0.0 : mn;     /* Math.max(0, ...) */
            }
}

static void *pool_worker(void *arg) {
    jpool *j = (jpool *)arg;
    const jplan *p = j->p;
    double *cache = (double *)malloc(sizeof(double) * (p->n_sums + 1));
    unsigned char *have = (unsigned char *)malloc((size_t)p->n_sums + 1);
    double *nzv = (double *)malloc(sizeof(double) * p->cs);
    int *nzi = (int *)malloc(sizeof(int) * p->cs);
    const int bx_n = j->W / p->cw, by_n = j->H / p->ch;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int c = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (c >= j->n_cubes) break;
        /* Transform.java:94-100 submission order: z outer, y, x inner */
        int bx = c % bx_n, by = (c / bx_n) % by_n, bz = c / (bx_n * by_n);
        if (j->kind == 0)
            dct_apply(p, (const uint8_t *)j->in, j->out, j->W, j->H, bx * p->cw, by * p->ch, bz * p->cd, cache, have);
        else
            idct_apply(p, (const double *)j->in, j->out, j->W, j->H, bx * p->cw, by * p->ch, bz * p->cd, nzv, nzi);
    }
    free(cache); free(have); free(nzv); free(nzi);
    return NULL;
}

static void run_pool(const jplan *p, const void *in, double *out, int W, int H, int F, int threads, int kind) {
    jpool j;
    j.p = p; j.in = in; j.out = out; j.W = W; j.H = H; j.F = F; j.kind = kind;
    j.n_cubes = (W / p->cw) * (H / p->ch) * (F / p->cd);
    j.next = 0;
    pthread_mutex_init(&j.mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, pool_worker, &j);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    free(th);
    pthread_mutex_destroy(&j.mu);
}

/* DCT over a raster stack (W x H x F frames, F multiple of cd).  out: double raster, zeroed here
   (Encoder.java:51 allocates a fresh double[]). */
void oracle_dct_forward(const jplan *p, const uint8_t *raster, int W, int H, int F, double *out, int threads) {
    memset(out, 0, sizeof(double) * (size_t)W * H * F);
    run_pool(p, raster, out, W, H, F, threads, 0);
}

void oracle_dct_inverse(const jplan *p, const double *coef_raster, int W, int H, int F, double *out, int threads) {
    memset(out, 0, sizeof(double) * (size_t)W * H * F);
    run_pool(p, coef_raster, out, W, H, F, threads, 1);
}

/* Encoder.java:75-89: raster DCT -> cube-major quantised (Math.round) */
void oracle_quantize(const double *dct, int W, int H, int F, int cw, int ch, int cd, int32_t *q) {
    size_t o = 0;
    const size_t frameSize = (size_t)W * H;
    for (int z = 0; z < F; z += cd)
        for (int y = 0; y < H; y += ch)
            for (int x = 0; x < W; x += cw)
                for (int k = 0; k < cd; k++)
                    for (int i = 0; i < ch; i++)
                        for (int j = 0; j < cw; j++) {
                            size_t pos = (size_t)(z + k) * frameSize + (size_t)(y + i) * W + x + j;
                            int st = 5 * (i + j + k);
                            if (st < 1) st = 1;
                            q[o++] = (int32_t)oracle_java_round(dct[pos] / (double)st);
                        }
}

/* Decoder.java:78-96: cube-major quantised -> raster dequantised doubles */
void oracle_dequantize(const int32_t *q, int W, int H, int F, int cw, int ch, int cd, double *out) {
    size_t o = 0;
    const size_t frameSize = (size_t)W * H;
    for (int z = 0; z < F; z += cd)
        for (int y = 0; y < H; y += ch)
            for (int x = 0; x < W; x += cw)
                for (int k = 0; k < cd; k++)
                    for (int i = 0; i < ch; i++)
                        for (int j = 0; j < cw; j++) {
                            size_t pos = (size_t)(z + k) * frameSize + (size_t)(y + i) * W + x + j;
                            int st = 5 * (i + j + k);
                            if (st < 1) st = 1;
                            out[pos] = (double)oracle_java_round((double)q[o++] * (double)st);
                        }
}

/* Decoder.java:112: (byte) videoPixels[i]  (double -> int truncation -> low 8 bits) */
void oracle_to_bytes(const double *v, size_t n, uint8_t *out) {
    for (size_t i = 0; i < n; i++) {
        double d = v[i];
        int32_t iv;
        if (d != d) iv = 0;
        else if (d >= 2147483647.0) iv = INT32_MAX;
        else if (d <= -2147483648.0) iv = INT32_MIN;
        else iv = (int32_t)d;
        out[i] = (uint8_t)(iv & 0xFF);
    }
}

/* Convenience: the full Java encode hot path (DCT + quantise) and decode hot path. */
void oracle_encode_q(const jplan *p, const uint8_t *raster, int W, int H, int F, int32_t *q, double *dct_out, int threads) {
    double *d = dct_out ? dct_out : (double *)malloc(sizeof(double) * (size_t)W * H * F);
    oracle_dct_forward(p, raster, W, H, F, d, threads);
    oracle_quantize(d, W, H, F, p->cw, p->ch, p->cd, q);
    if (!dct_out) free(d);
}

void oracle_decode_q(const jplan *p, const int32_t *q, int W, int H, int F, uint8_t *raster, int threads) {
    size_t n = (size_t)W * H * F;
    double *c = (double *)malloc(sizeof(double) * n);
    double *v = (double *)malloc(sizeof(double) * n);
    oracle_dequantize(q, W, H, F, p->cw, p->ch, p->cd, c);
    oracle_dct_inverse(p, c, W, H, F, v, threads);
    oracle_to_bytes(v, n, raster);
    free(c); free(v);
}

/* ------------------------------------------------------------------------------------------ */
/* CubeUtils.diagonalSlices (CubeUtils.java:7-41); positions as (x,y,z) triples               */
/* ------------------------------------------------------------------------------------------ */
int oracle_diagonal_slices(int width, int height, int depth, int32_t *xyz) {
    int n = 0;
    int maxSum = (width - 1) + (height - 1) + (depth - 1);
    for (int t = 0; t <= maxSum; t++) {
        int maxW = (width - 1) < t ? (width - 1) : t;
        int maxH = (height - 1) < t ? (height - 1) : t;
        int maxD = (depth - 1) < t ? (depth - 1) : t;
        int minW = t - (maxH + maxD); if (minW < 0) minW = 0;
        int minH = t - (maxW + maxD); if (minH < 0) minH = 0;
        int minD = t - (maxH + maxW); if (minD < 0) minD = 0;
        for (int y = minH; y <= maxH; y++)
            for (int z = minD; z <= maxD; z++)
                for (int x = minW; x <= maxW; x++)
                    if (x + y + z == t) {
                        xyz[3 * n] = x; xyz[3 * n + 1] = y; xyz[3 * n + 2] = z;
                        n++;
                    }
    }
    return n;
}

/* ------------------------------------------------------------------------------------------ */
/* ExpGolombWriter / ExpGolombReader (Java semantics; byte[] is zero-initialised)               */
/* ------------------------------------------------------------------------------------------ */
static int eg_bits(int v) { int c = 0; while (v != 0) { v = v >> 1; c++; } return c; }
static int eg_mask(int b) { int m = 0; while (b > 0) { m = (m << 1) | 1; b--; } return m; }

/* Writes n values; returns getBufferPosition() (the Java encoder deflates pos+1 bytes).
   buf must be zeroed and large enough. */
int oracle_eg_write(const int32_t *vals, size_t n, uint8_t *buf) {
    int bitPosition = 8, bufferPosition = 0;
    for (size_t i = 0; i < n; i++) {
        int value = vals[i];
        if (value <= 0) value = -2 * value; else value = 2 * value - 1;
        value += 1;
        int bitsCount = eg_bits(value);
        int mask = eg_mask(bitsCount);
        int zeroes = bitsCount - 1;
        bitPosition -= zeroes;
        while (bitPosition <= 0) { bufferPosition += 1; bitPosition += 8; }
        while (bitsCount > 0) {
            if (bitPosition > bitsCount) {
                buf[bufferPosition] = (uint8_t)(buf[bufferPosition] | (value << (bitPosition - bitsCount)));
                bitPosition -= bitsCount;
                bitsCount = 0;
            } else {
                int reduced = value >> (bitsCount - bitPosition);
                buf[bufferPosition] = (uint8_t)(buf[bufferPosition] | reduced);
                bitsCount -= bitPosition;
                mask = mask >> bitPosition;
                bufferPosition += 1;
                bitPosition = 8;
                value = value & mask;
            }
        }
    }
    return bufferPosition;
}

/* Reads n values (ExpGolombReader.readValue); returns bytes consumed position. */
int oracle_eg_read(const uint8_t *buf, size_t buflen, size_t n, int32_t *out) {
    int bitPosition = 8;
    size_t bufferPosition = 0;
#define EGB(i) ((int)(int8_t)((i) < buflen ? buf[(i)] : 0))
    for (size_t v = 0; v < n; v++) {
        int zeroes = 0;
        int byteValue = EGB(bufferPosition);
        int bit = byteValue & (1 << (bitPosition - 1));
        while (bit == 0) {
            zeroes++;
            bitPosition--;
            if (bitPosition <= 0) { bufferPosition++; bitPosition = 8; byteValue = EGB(bufferPosition); }
            bit = byteValue & (1 << (bitPosition - 1));
            if (bufferPosition > buflen + 8) return -1;
        }
        int value = 0, bitCount = zeroes + 1;
        while (bitCount > 0) {
            if (bitCount > bitPosition) {
                int mask = eg_mask(bitPosition);
                value = value | ((byteValue & mask) << (bitCount - bitPosition));
                bitCount -= bitPosition;
                bitPosition = 8;
                bufferPosition += 1;
                byteValue = EGB(bufferPosition);
            } else {
                int mask = eg_mask(bitCount) << (bitPosition - bitCount);
                value = value | ((byteValue & mask) >> (bitPosition - bitCount));
                bitPosition -= bitCount;
                bitCount = 0;
                if (bitPosition <= 0) { bitPosition = 8; bufferPosition += 1; byteValue = EGB(bufferPosition); }
            }
        }
        value -= 1;
        if (value % 2 != 0) value = (value + 1) / 2; else value = -value / 2;
        out[v] = value;
    }
#undef EGB
    return (int)bufferPosition;
}
