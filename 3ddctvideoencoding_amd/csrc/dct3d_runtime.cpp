// dct3d_runtime.cpp -- the C-ABI (include/dct3d.h): context, buffers, launches.
//
// Replaces the reference's per-call OpenCL setup (encoder.c:147-197, decoder.c:153-202,
// OpenCLUtils.c:49-165) with a persistent context: the transform plan (DCT.initialize equivalent,
// dct3d_plan.cpp) is built once and its fold tables uploaded once; device work buffers are grown on
// demand and reused; everything runs on one HIP stream.  Errors are returned, never printed, never
// exit()ed (the reference exit(1)s inside OpenCLUtils.c:40-162).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <vector>
#include <cstring>
#include <mutex>
#include <condition_variable>
#include <deque>
#include <thread>
#include <new>

#include "../../include/dct3d.h"
#include "dct3d_kernels.h"
#include "dct3d_plan.h"

using namespace dct3d;

namespace {

// the stream decode's status words (d_egd_status): [0, 4) the sync / mark passes' (EgDecParams::status),
// [4, 6) the chunk scan's (EgParams::status)
constexpr size_t kEgdStatusBytes = 6 * sizeof(uint64_t);

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int grow(size_t need) {
        if (need <= bytes) return DCT3D_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, need) != hipSuccess) return DCT3D_ENOMEM;
        bytes = need;
        return DCT3D_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

}  // namespace

struct dct3d_ctx {
    int device = 0;
    int bw = 8, bh = 8, bd = 8;
    Plan plan;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    bool profiling = false;
    // ring of event quadruples (main kernel begin/end, auxiliary launch begin/end); resolved lazily
    static constexpr int kRing = 256;
    hipEvent_t ev[kRing][4] = {};
    int ring_head = 0, ring_pending = 0;
    uint64_t n_timed = 0;
    double kernel_ms = 0.0, aux_ms = 0.0;
    // plan tables on device
    DevBuf d_ngroups, d_coef, d_group_of, d_inv_coef, d_tabs, d_tabs64;
    // test / diagnostic options (dct3d_ctx_set_option): how later calls reach their results
    double opt_dec_margin = 0.0;    // added to the decode margin
    bool opt_enc_no_recheck = false, opt_eg_two_step = false,
         opt_eg_no_resolve = false;
    bool opt_eg_force_retry = false;
    bool opt_eg_fused_front = false;
    int opt_eg_dec_groups = 0;  // fused stream decode: groups per wave (0: the default, 8)
    // certify-or-replay state
    uint64_t last_units = 0;
    bool last_valid = false;
    // in-wave replay (encode, decode): two counter slots that alternate between calls; each launch zeroes
    // the other slot for the next call, so a call needs no reset copy (zeroed once at creation).
    // Slot j (2 kCountSpread words at j * 2 kCountSpread): Java-fold replays, then second-certificate
    // settlements, each spread over kCountSpread words (dct3d_kernels.h).
    DevBuf d_enc_counts;
    int enc_slot = 0;
    int last_count_slot = -1;  // >= 0: the last call's statistics are in d_enc_counts[slot]
    bool slot_used = false;    // a counting kernel of the current call was enqueued into enc_slot
    bool batch = false;        // a host entry point's chunks: one slot for the whole call (batch_end flips it)
    uint64_t batch_units = 0;
    hipEvent_t ev_switch = nullptr;  // orders a dct3d_ctx_set_stream switch after the old stream's work
    // host-pointer entry point staging
    DevBuf h_in, h_out, h_aux;
    // Exp-Golomb stage: diagonal order, per-cube bits / offsets, chunk sums, status, device stream
    DevBuf d_diag, d_eg_bits, d_eg_off, d_eg_bsum, d_eg_status, d_eg_out, d_eg_q, d_eg_ht;
    // fused encode + Exp-Golomb: per-segment slots and lane bit counts
    DevBuf d_egf_slot;
    // Exp-Golomb decode: chunk exits (two passes' worth), decode status, staged stream / raster
    // (d_egd_status: the decode's four status words, then the scan's two -- one read-back per call)
    DevBuf d_egd_exit, d_egd_status, d_egd_in, d_egd_raster, d_egd_mark, d_egd_desc;
    // d_egd_status holds two slots of the words; calls alternate between them, and the fused decode's
    // consumer zeroes the other slot for the next call (clean: known zero, no memset needed)
    int egd_slot = 0;
    bool egd_clean[2] = {true, true};
    // the same for the encode stream's two status words (d_eg_status: two slots of 16 bytes)
    int eg_slot = 0;
    bool eg_clean[2] = {true, true};
    // pinned host words the entropy stages' status lands in (one DMA read-back, not a pageable copy)
    uint64_t* h_status = nullptr;
    uint64_t* h_status_dev = nullptr;  // its device-side address (decode_eg_kernel writes the words there)
    uint64_t egd_seq = 0;              // stream-decode calls so far: decode_eg_kernel's hand-off tag (h_status[6])
    uint64_t eg_seq = 0;               // stream-encode calls so far: eg_stitch_kernel's hand-off tag (h_status[7])
    // host-pointer pipeline: copy streams, slot events, double-buffered slots
    hipStream_t s_up = nullptr, s_down = nullptr;
    hipEvent_t pe_in[2] = {}, pe_done[2] = {};
    DevBuf p_in[2], p_out[2];
    uint64_t eg_last_bytes = 0;
};

// diagonal-slice order (CubeUtils.c:5-46): x + y + z ascending; y outer, z middle, x inner
static int diagonal_order(int bw, int bh, int bd, uint16_t* out) {
    int n = 0;
    for (int t = 0; t <= (bw - 1) + (bh - 1) + (bd - 1); t++)
        for (int y = 0; y <= (bh - 1 < t ? bh - 1 : t); y++)
            for (int z = 0; z <= (bd - 1 < t ? bd - 1 : t); z++) {
                const int x = t - y - z;
                if (x < 0 || x > bw - 1) continue;
                out[n++] = (uint16_t)(x + bw * y + bw * bh * z);
            }
    return n;
}

// FastDiv of the kernel params (dct3d_kernels.h): s = 31 + ceil(log2 d), m = ceil(2^s / d)
static FastDiv fast_div(uint32_t d) {
    uint32_t l = 0;
    while ((1ull << l) < d) l++;
    FastDiv f;
    f.s = 31 + l;
    f.m = (uint32_t)(((1ull << f.s) + d - 1) / d);
    return f;
}
template <class T>
static void set_fast_div(T& P) {
    P.div_cps = fast_div(P.cubes_per_stack);
    P.div_nbx = fast_div(P.nbx);
}

extern "C" {

int dct3d_abi_version(void) { return DCT3D_ABI_VERSION; }

const char* dct3d_strerror(int code) {
    switch (code) {
        case DCT3D_OK: return "ok";
        case DCT3D_EINVAL: return "invalid argument";
        case DCT3D_EDEVICE: return "HIP device error";
        case DCT3D_ENOMEM: return "out of memory";
        case DCT3D_EKERNEL: return "kernel launch failed";
        case DCT3D_ENOSPC: return "output buffer too small";
        case DCT3D_ENODATA: return "input stream ends early";
        default: return "unknown error";
    }
}

// the status words of an entropy stage (device, written by its kernels on the context stream): one
// asynchronous copy into the pinned words, then the stream's completion
// The end of a synchronous call: the stream polled for a while before blocking (a blocking wait took
// ~15-40 us to return after the stream's last kernel, profiles/r06/gaps/), so that the caller's next
// call reaches the device sooner.
static int stream_wait(dct3d_ctx* c) {
    for (int i = 0; i < 20000; i++) {
        const hipError_t e = hipStreamQuery(c->stream);
        if (e == hipSuccess) return DCT3D_OK;
        if (e != hipErrorNotReady) return DCT3D_EDEVICE;
    }
    return hipStreamSynchronize(c->stream) == hipSuccess ? DCT3D_OK : DCT3D_EDEVICE;
}
static int read_status(dct3d_ctx* c, const void* d_status, size_t bytes, uint64_t* out) {
    if (hipMemcpyAsync(c->h_status, d_status, bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        stream_wait(c))
        return DCT3D_EDEVICE;
    memcpy(out, c->h_status, bytes);
    return DCT3D_OK;
}

// The encode stream's status words for this call (zeroed: by a memset unless the last call's stitch kernel
// cleared this slot), and the kernel-side hand-off (EgParams::status_host / status_clear).
static uint64_t* eg_status_begin(dct3d_ctx* c, int* rc) {
    uint64_t* st = (uint64_t*)c->d_eg_status.p + 2 * c->eg_slot;
    const bool clean = c->eg_clean[c->eg_slot];
    c->eg_clean[c->eg_slot] = false;
    *rc = !clean && hipMemsetAsync(st, 0, 16, c->stream) != hipSuccess ? DCT3D_EDEVICE : DCT3D_OK;
    return st;
}
static void eg_status_handoff(dct3d_ctx* c, EgParams& P) {
    P.status_host = c->h_status_dev;
    P.status_clear = (uint64_t*)c->d_eg_status.p + 2 * (c->eg_slot ^ 1);
    P.seq = ++c->eg_seq;
}
static int wait_tag(dct3d_ctx* c, int word, uint64_t seq, uint64_t* value, uint32_t* flags);
// after the stitch kernel was enqueued with the hand-off: the call returns when the stitch's block 0 has
// handed the verdict over (the tag), the stitch's last words completing on the stream (a wait for the
// stream's end instead took ~30 us longer to return, profiles/r06/gaps/timed)
static int eg_status_end(dct3d_ctx* c, bool handoff, const uint64_t* st, uint64_t* out, uint64_t seq = 0) {
    int rc;
    if (handoff) {
        c->eg_clean[c->eg_slot ^ 1] = true;
        uint64_t v = 0;
        uint32_t fl = 0;
        rc = wait_tag(c, 7, seq, &v, &fl);
        if (!rc && (fl & kTagOverflow)) {  // the total did not fit the tag: the words, after the stream
            rc = stream_wait(c);
            if (!rc) memcpy(out, c->h_status, 16);
        } else if (!rc) {
            out[0] = v;
            out[1] = fl & 3u;
        }
    } else {
        rc = read_status(c, st, 16, out);
    }
    c->eg_slot ^= 1;
    return rc;
}

static int upload(DevBuf& b, const void* src, size_t bytes) {
    int rc = b.grow(bytes);
    if (rc) return rc;
    return hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? DCT3D_OK : DCT3D_EDEVICE;
}

int dct3d_plan_query(int bw, int bh, int bd, dct3d_plan_info* info, int32_t* ngroups, double* coef,
                     uint8_t* group_of, double* enc_K) {
    Plan p;
    if (!build_plan(bw, bh, bd, p)) return DCT3D_EINVAL;
    if (info) {
        memset(info, 0, sizeof(*info));
        info->cube_size = p.cs;
        info->n_mults = p.n_mults;
        info->treeified = p.treeified ? 1 : 0;
        info->coef_dc = p.coef_dc;
        info->dec_G = p.dec_G;
        info->dec_E = p.dec_E;
        info->dec_l1_max = p.dec_l1_max;
        memcpy(info->enc_rstep, p.enc_rstep, sizeof(info->enc_rstep));
        memcpy(info->enc_G, p.enc_G, sizeof(info->enc_G));
        memcpy(info->enc_E, p.enc_E, sizeof(info->enc_E));
        memcpy(info->enc_thr64, p.enc_thr64, sizeof(info->enc_thr64));
    }
    if (ngroups) memcpy(ngroups, p.fwd_ngroups.data(), sizeof(int32_t) * p.cs);
    if (coef) memcpy(coef, p.fwd_coef.data(), sizeof(double) * p.fwd_coef.size());
    if (group_of) memcpy(group_of, p.fwd_group_of.data(), p.fwd_group_of.size());
    if (enc_K) memcpy(enc_K, p.enc_K.data(), sizeof(double) * p.cs);
    return DCT3D_OK;
}

int dct3d_ctx_create(int device, int block_w, int block_h, int block_d, dct3d_ctx** out) {
    if (!out) return DCT3D_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return DCT3D_EDEVICE;
    dct3d_ctx* c = new (std::nothrow) dct3d_ctx();
    if (!c) return DCT3D_ENOMEM;
    c->device = device;
    c->bw = block_w;
    c->bh = block_h;
    c->bd = block_d;
    if (!build_plan(block_w, block_h, block_d, c->plan)) {
        delete c;
        return DCT3D_EINVAL;
    }
    // the context's own stream is a blocking stream: ordered with the legacy default stream, so device
    // buffers a caller fills or reads there (e.g. a framework's default stream) need no extra sync
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamDefault) != hipSuccess) {
        delete c;
        return DCT3D_EDEVICE;
    }
    c->stream = c->own_stream;
    for (auto& q : c->ev)
        for (auto& e : q)
            if (hipEventCreate(&e) != hipSuccess) {
                dct3d_ctx_destroy(c);
                return DCT3D_EDEVICE;
            }
    const Plan& p = c->plan;
    float tabs[3 * kMaxS];
    memcpy(tabs, p.enc_rstep, sizeof(float) * kMaxS);
    memcpy(tabs + kMaxS, p.enc_G, sizeof(float) * kMaxS);
    memcpy(tabs + 2 * kMaxS, p.enc_E, sizeof(float) * kMaxS);
    int rc = upload(c->d_ngroups, p.fwd_ngroups.data(), p.fwd_ngroups.size() * sizeof(int32_t));
    if (!rc) rc = upload(c->d_coef, p.fwd_coef.data(), p.fwd_coef.size() * sizeof(double));
    if (!rc) rc = upload(c->d_group_of, p.fwd_group_of.data(), p.fwd_group_of.size());
    if (!rc) {  // transposed, [k][n]: the replay kernel's threads (one per pixel n) read it coalesced
        std::vector<double> t(p.inv_coef.size());
        for (int n = 0; n < p.cs; n++)
            for (int k = 0; k < p.cs; k++) t[(size_t)k * p.cs + n] = p.inv_coef[(size_t)n * p.cs + k];
        rc = upload(c->d_inv_coef, t.data(), t.size() * sizeof(double));
    }
    if (!rc) rc = upload(c->d_tabs, tabs, sizeof(tabs));
    if (!rc) {  // second certificate (8x8x8): [64] fp64 basis, [32] thresholds
        double t64[64 + kMaxS];
        memcpy(t64, p.basis64, sizeof(p.basis64));
        memcpy(t64 + 64, p.enc_thr64, sizeof(p.enc_thr64));
        rc = upload(c->d_tabs64, t64, sizeof(t64));
    }
    if (!rc) rc = c->d_enc_counts.grow(4 * kCountSpread * sizeof(uint32_t));
    if (!rc && hipMemset(c->d_enc_counts.p, 0, 4 * kCountSpread * sizeof(uint32_t)) != hipSuccess) rc = DCT3D_EDEVICE;
    if (!rc) {
        std::vector<uint16_t> diag(p.cs);
        diagonal_order(block_w, block_h, block_d, diag.data());
        rc = upload(c->d_diag, diag.data(), diag.size() * sizeof(uint16_t));
    }
    if (!rc) rc = c->d_eg_status.grow(32);
    if (!rc && hipMemset(c->d_eg_status.p, 0, 32) != hipSuccess) rc = DCT3D_EDEVICE;
    if (!rc) rc = c->d_egd_status.grow(2 * kEgdStatusBytes);
    if (!rc && hipMemset(c->d_egd_status.p, 0, 2 * kEgdStatusBytes) != hipSuccess) rc = DCT3D_EDEVICE;
    if (!rc && hipHostMalloc((void**)&c->h_status, kEgdStatusBytes + 16, hipHostMallocDefault) != hipSuccess) {
        c->h_status = nullptr;
        rc = DCT3D_ENOMEM;
    }
    if (!rc) memset(c->h_status, 0, kEgdStatusBytes + 16);
    if (!rc && hipHostGetDevicePointer((void**)&c->h_status_dev, c->h_status, 0) != hipSuccess) c->h_status_dev = nullptr;
    if (rc) {
        dct3d_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return DCT3D_OK;
}

void dct3d_ctx_destroy(dct3d_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    for (DevBuf* b : {&c->d_ngroups, &c->d_coef, &c->d_group_of, &c->d_inv_coef, &c->d_tabs, &c->d_tabs64,
                      &c->d_enc_counts, &c->h_in, &c->h_out, &c->h_aux, &c->d_diag, &c->d_eg_bits,
                      &c->d_eg_off, &c->d_eg_bsum, &c->d_eg_status, &c->d_eg_out, &c->d_eg_q, &c->d_eg_ht,
                      &c->d_egd_exit, &c->d_egd_status, &c->d_egd_in, &c->d_egd_raster, &c->d_egd_mark, &c->d_egd_desc,
                      &c->d_egf_slot})
        b->release();
    if (c->h_status) (void)hipHostFree(c->h_status);
    for (auto& q : c->ev)
        for (auto& e : q)
            if (e) (void)hipEventDestroy(e);
    if (c->s_up) (void)hipStreamDestroy(c->s_up);
    if (c->s_down) (void)hipStreamDestroy(c->s_down);
    for (int i = 0; i < 2; i++) {
        if (c->pe_in[i]) (void)hipEventDestroy(c->pe_in[i]);
        if (c->pe_done[i]) (void)hipEventDestroy(c->pe_done[i]);
    }
    if (c->ev_switch) (void)hipEventDestroy(c->ev_switch);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int dct3d_ctx_set_stream(dct3d_ctx* c, void* s) {
    if (!c) return DCT3D_EINVAL;
    const hipStream_t ns = s ? (hipStream_t)s : c->own_stream;
    if (ns != c->stream) {
        // work enqueued on the new stream runs after the old stream's: a later launch would otherwise
        // overlap an earlier one whose block 0 clears the counter slot the later one counts into
        if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
        if (!c->ev_switch && hipEventCreateWithFlags(&c->ev_switch, hipEventDisableTiming) != hipSuccess)
            return DCT3D_EDEVICE;
        if (hipEventRecord(c->ev_switch, c->stream) == hipSuccess) {
            if (hipStreamWaitEvent(ns, c->ev_switch, 0) != hipSuccess) return DCT3D_EDEVICE;
        } else {
            // HIP rejected the old handle (a caller's stream destroyed before the switch, against the
            // contract in dct3d.h): order by a device-wide synchronisation.  A destroyed handle that HIP
            // has reused for a new stream is not detectable here -- hence the contract.
            (void)hipGetLastError();
            if (hipDeviceSynchronize() != hipSuccess) return DCT3D_EDEVICE;
        }
    }
    c->stream = ns;
    return DCT3D_OK;
}

int dct3d_ctx_info(const dct3d_ctx* c, int* device, int* block_d, void** hip_stream) {
    if (!c) return DCT3D_EINVAL;
    if (device) *device = c->device;
    if (block_d) *block_d = c->bd;
    if (hip_stream) *hip_stream = (void*)c->stream;
    return DCT3D_OK;
}

int dct3d_ctx_set_option(dct3d_ctx* c, int option, double value) {
    if (!c || !(value >= 0.0)) return DCT3D_EINVAL;
    switch (option) {
        case DCT3D_OPT_DEC_MARGIN: c->opt_dec_margin = value; return DCT3D_OK;
        case DCT3D_OPT_ENC_NO_RECHECK: c->opt_enc_no_recheck = value != 0.0; return DCT3D_OK;
        case DCT3D_OPT_EG_TWO_STEP: c->opt_eg_two_step = value != 0.0; return DCT3D_OK;
        case DCT3D_OPT_EG_NO_RESOLVE: c->opt_eg_no_resolve = value != 0.0; return DCT3D_OK;
        case DCT3D_OPT_EG_FORCE_RETRY: c->opt_eg_force_retry = value != 0.0; return DCT3D_OK;
        case DCT3D_OPT_EG_FUSED_FRONT: c->opt_eg_fused_front = value != 0.0; return DCT3D_OK;
        case DCT3D_OPT_EG_DEC_GROUPS:
            if (value != 0.0 && value != 1.0 && value != 2.0 && value != 4.0 && value != 8.0) return DCT3D_EINVAL;
            c->opt_eg_dec_groups = (int)value;
            return DCT3D_OK;
        default: return DCT3D_EINVAL;
    }
}

int dct3d_ctx_set_profiling(dct3d_ctx* c, int on) {
    if (!c) return DCT3D_EINVAL;
    c->profiling = on != 0;
    return DCT3D_OK;
}

int dct3d_synchronize(dct3d_ctx* c) {
    if (!c) return DCT3D_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    return hipStreamSynchronize(c->stream) == hipSuccess ? DCT3D_OK : DCT3D_EDEVICE;
}

// Resolves the oldest `n` pending timing slots (their events have been recorded on the stream).
static int resolve_timers(dct3d_ctx* c, int n) {
    for (; n > 0 && c->ring_pending > 0; n--) {
        const int slot = (c->ring_head - c->ring_pending + dct3d_ctx::kRing) % dct3d_ctx::kRing;
        hipEvent_t* e = c->ev[slot];
        if (hipEventSynchronize(e[3]) != hipSuccess) return DCT3D_EDEVICE;
        float a = 0.f, b = 0.f;
        if (hipEventElapsedTime(&a, e[0], e[1]) != hipSuccess || hipEventElapsedTime(&b, e[2], e[3]) != hipSuccess)
            return DCT3D_EDEVICE;
        c->kernel_ms += a;
        c->aux_ms += b;
        c->n_timed++;
        c->ring_pending--;
    }
    return DCT3D_OK;
}

// Returns the event quadruple for this call (or nullptr when profiling is off).
static hipEvent_t* timing_slot(dct3d_ctx* c) {
    if (!c->profiling) return nullptr;
    if (c->ring_pending == dct3d_ctx::kRing && resolve_timers(c, 1)) return nullptr;
    hipEvent_t* e = c->ev[c->ring_head];
    c->ring_head = (c->ring_head + 1) % dct3d_ctx::kRing;
    c->ring_pending++;
    return e;
}

int dct3d_reset_timers(dct3d_ctx* c) {
    if (!c) return DCT3D_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    int rc = resolve_timers(c, dct3d_ctx::kRing);
    c->n_timed = 0;
    c->kernel_ms = c->aux_ms = 0.0;
    return rc;
}

int dct3d_get_stats(dct3d_ctx* c, dct3d_stats* st) {
    if (!c || !st) return DCT3D_EINVAL;
    memset(st, 0, sizeof(*st));
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (resolve_timers(c, dct3d_ctx::kRing)) return DCT3D_EDEVICE;
    st->n_timed = c->n_timed;
    st->kernel_ms_total = c->kernel_ms;
    st->aux_ms_total = c->aux_ms;
    st->n_units = c->last_units;
    if (!c->last_valid || c->last_count_slot < 0) return DCT3D_OK;
    // the call's counter slot (in-wave replays: every replaying path has one)
    std::vector<uint32_t> w(2 * kCountSpread);
    if (hipMemcpyAsync(w.data(), (uint32_t*)c->d_enc_counts.p + c->last_count_slot * 2 * kCountSpread,
                       w.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return DCT3D_EDEVICE;
    for (int i = 0; i < kCountSpread; i++) {
        st->n_flagged += w[i];
        st->n_rechecked += w[kCountSpread + i];
    }
    return DCT3D_OK;
}

// ---------------------------------------------------------------------------------------------
static int check_geometry(const dct3d_ctx* c, int w, int h, int n_stacks, uint64_t* n_cubes) {
    if (w <= 0 || h <= 0 || n_stacks < 0) return DCT3D_EINVAL;
    if (w % c->bw || h % c->bh) return DCT3D_EINVAL;  // the reference overruns silently here
    const uint64_t cps = (uint64_t)(w / c->bw) * (uint64_t)(h / c->bh);
    const uint64_t n = cps * (uint64_t)n_stacks;
    if (n >= (1ull << 31) / 8) return DCT3D_EINVAL;   // 32-bit cube indices in the kernels
    *n_cubes = n;
    return DCT3D_OK;
}

// Decode: uncertified cubes are replayed inside the wave; the replay count goes to the ctx's current
// counter slot, and the launch zeroes the other one for the next call (see d_enc_counts).
static void set_count_slot(dct3d_ctx* c, unsigned int*& count, unsigned int*& clear) {
    count = (unsigned int*)c->d_enc_counts.p + c->enc_slot * 2 * kCountSpread;
    clear = (unsigned int*)c->d_enc_counts.p + (c->enc_slot ^ 1) * 2 * kCountSpread;
}
static void set_dec_replay(dct3d_ctx* c, DecodeParams& P) {
    P.inv_coef_t = (const double*)c->d_inv_coef.p;
    set_count_slot(c, P.replay_count, P.replay_clear);
}
// A call's counting kernels are enqueued: its statistics are in enc_slot (units of work: `units`).  The
// slot flips at the end of the call -- of every chunk together inside a host entry point's pipeline
// (batch), and whenever a counting kernel was enqueued, even if a later step of the call failed (the
// next call must start on the slot this one's launches zeroed).
static void count_slot_used(dct3d_ctx* c, uint64_t units) {
    c->slot_used = true;
    if (c->batch) {
        c->batch_units += units;
        return;
    }
    c->last_count_slot = c->enc_slot;
    c->enc_slot ^= 1;
    c->slot_used = false;
    c->last_units = units;
    c->last_valid = true;
}
static void batch_begin(dct3d_ctx* c) {
    c->batch = true;
    c->batch_units = 0;
    c->slot_used = false;
    c->last_valid = false;
    c->last_count_slot = -1;
}
static void batch_end(dct3d_ctx* c) {
    c->batch = false;
    if (!c->slot_used) return;
    c->last_count_slot = c->enc_slot;
    c->enc_slot ^= 1;
    c->slot_used = false;
    c->last_units = c->batch_units;
    c->last_valid = true;
}

static int forward_f64_raster(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, uint64_t n_cubes, double* d_out) {
    Fwd64Params P;
    P.raster = d_raster;
    P.out = d_out;
    P.n_cubes = (uint32_t)n_cubes;
    P.cubes_per_stack = (uint32_t)((w / 8) * (h / 8));
    P.nbx = (uint32_t)(w / 8);
    P.width = (uint32_t)w;
    P.plane = (uint64_t)w * h;
    P.stack_stride = P.plane * c->bd;
    return launch_fwd64_raster(c->bd, P, c->stream) ? DCT3D_EKERNEL : DCT3D_OK;
}

int dct3d_encode_stacks_dev(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, int n_stacks, int32_t* d_q,
                            double* d_dct) {
    if (!c || (!d_raster && n_stacks) || (!d_q && n_stacks)) return DCT3D_EINVAL;
    uint64_t n_cubes;
    int rc = check_geometry(c, w, h, n_stacks, &n_cubes);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (!c->batch) {
        c->last_valid = false;
        c->last_count_slot = -1;
    }
    if (n_cubes == 0) return DCT3D_OK;
    const int D = c->bd;
    // one launch: uncertified coefficients are replayed inside the wave (exact Java fold)
    const uint64_t plane = (uint64_t)w * h;
    EncodeParams P;
    memset(&P, 0, sizeof(P));
    P.raster = d_raster;
    P.out = d_q;
    P.n_cubes = (uint32_t)n_cubes;
    P.g_base = 0;
    P.cubes_per_stack = (uint32_t)((w / 8) * (h / 8));
    P.nbx = (uint32_t)(w / 8);
    set_fast_div(P);
    P.width = (uint32_t)w;
    P.plane = plane;
    P.stack_stride = plane * D;
    P.coef_dc = c->plan.coef_dc;
    const float* tabs = (const float*)c->d_tabs.p;
    P.tab_rstep = tabs;
    P.tab_G = tabs + kMaxS;
    P.tab_E = tabs + 2 * kMaxS;
    P.ngroups = (const int32_t*)c->d_ngroups.p;
    P.coef = (const double*)c->d_coef.p;
    P.group_of = (const uint8_t*)c->d_group_of.p;
    set_count_slot(c, P.replay_count, P.replay_clear);
    P.tab64 = (const double*)c->d_tabs64.p;
    P.recheck = c->opt_enc_no_recheck ? 0u : 1u;
    hipEvent_t* ev = timing_slot(c);
    if (ev) (void)hipEventRecord(ev[0], c->stream);
    if (launch_encode(D, P, c->stream)) return DCT3D_EKERNEL;
    if (ev) {  // single launch: the second event pair brackets nothing
        (void)hipEventRecord(ev[1], c->stream);
        (void)hipEventRecord(ev[2], c->stream);
        (void)hipEventRecord(ev[3], c->stream);
    }
    count_slot_used(c, n_cubes * (uint64_t)c->plan.cs);
    if (d_dct) return forward_f64_raster(c, d_raster, w, h, n_cubes, d_dct);
    return DCT3D_OK;
}

int dct3d_decode_stacks_dev(dct3d_ctx* c, const int32_t* d_q, int w, int h, int n_stacks, uint8_t* d_raster) {
    if (!c || (!d_raster && n_stacks) || (!d_q && n_stacks)) return DCT3D_EINVAL;
    uint64_t n_cubes;
    int rc = check_geometry(c, w, h, n_stacks, &n_cubes);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (!c->batch) {
        c->last_valid = false;
        c->last_count_slot = -1;
    }
    if (n_cubes == 0) return DCT3D_OK;
    const int D = c->bd;
    const uint64_t plane = (uint64_t)w * h;
    DecodeParams P;
    P.in = d_q;
    P.out = d_raster;
    P.n_cubes = (uint32_t)n_cubes;
    P.cube_base = 0;
    P.cubes_per_stack = (uint32_t)((w / 8) * (h / 8));
    P.nbx = (uint32_t)(w / 8);
    set_fast_div(P);
    P.width = (uint32_t)w;
    P.plane = plane;
    P.stack_stride = plane * D;
    P.dec_G = c->plan.dec_G;
    P.dec_E = c->plan.dec_E;
    P.dec_l1_max = c->plan.dec_l1_max;
    P.blk_store = (w / 8) % 2 == 0 && plane * D < (1ull << 32) ? 1u : 0u;  // dec_store_tile's conditions
    // test option: widen the certification margin so that most pixels are uncertified and their cubes
    // take the whole-cube replay path (tests/test_gpu_parity.py); a wider margin is never unsafe
    P.dec_E += c->opt_dec_margin;
    set_dec_replay(c, P);
    hipEvent_t* ev = timing_slot(c);
    if (ev) (void)hipEventRecord(ev[0], c->stream);
    if (launch_decode(D, P, c->stream)) return DCT3D_EKERNEL;
    if (ev) {  // one launch: the second event pair brackets nothing
        (void)hipEventRecord(ev[1], c->stream);
        (void)hipEventRecord(ev[2], c->stream);
        (void)hipEventRecord(ev[3], c->stream);
    }
    count_slot_used(c, n_cubes * (uint64_t)c->plan.cs);
    return DCT3D_OK;
}

// ---- host-pointer pipeline ------------------------------------------------------
// The host entry points move whole stacks in chunks: chunk i's upload (copy stream s_up, issued here),
// its kernels (the context stream, after the upload's event) and its download (copy stream s_down,
// issued by a helper thread: a D2H copy into pageable memory blocks the thread that issues it) overlap
// with chunk i+1's upload and chunk i-1's download.  PCIe is full duplex (~57 GB/s each way measured,
// pinned or pageable), so a call approaches max(in, out) / link rate instead of (in + out) / rate.
// Two device slots per direction; chunk i reuses slot i & 1 after chunk i-2's kernels (event) and
// download (the helper has returned from it) are done.  Synchronous on return, like the reference.
}  // extern "C" (the pipeline helpers are C++ templates)
static int ensure_pipe(dct3d_ctx* c) {
    if (c->s_up) return DCT3D_OK;
    if (hipStreamCreateWithFlags(&c->s_up, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->s_down, hipStreamNonBlocking) != hipSuccess)
        return DCT3D_EDEVICE;
    for (int i = 0; i < 2; i++)
        if (hipEventCreateWithFlags(&c->pe_in[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->pe_done[i], hipEventDisableTiming) != hipSuccess)
            return DCT3D_EDEVICE;
    return DCT3D_OK;
}

static int chunk_stacks_for(size_t bytes_per_stack, int n_stacks) {
    // ~64 MB per chunk on the heavier side, at least 1 stack, at most n_stacks / 2 (some overlap)
    size_t k = (64u << 20) / (bytes_per_stack ? bytes_per_stack : 1);
    if (k < 1) k = 1;
    const int half = n_stacks > 1 ? (n_stacks + 1) / 2 : 1;
    return (int)(k < (size_t)half ? k : (size_t)half);
}

// compute(d_in, d_out, first_stack, stacks) enqueues one chunk's kernels on c->stream; align: chunks of a
// multiple of this many stacks (the last one ragged)
template <class Compute>
static int run_pipeline(dct3d_ctx* c, int n_stacks, size_t in_per_stack, size_t out_per_stack, const void* host_in,
                        void* host_out, Compute&& compute, int align = 1) {
    int rc = ensure_pipe(c);
    if (rc) return rc;
    int cst = chunk_stacks_for(in_per_stack > out_per_stack ? in_per_stack : out_per_stack, n_stacks);
    cst = (cst + align - 1) / align * align;
    const int n_chunks = (n_stacks + cst - 1) / cst;
    for (int s = 0; s < 2; s++)
        if ((in_per_stack && (rc = c->p_in[s].grow(cst * in_per_stack))) || (rc = c->p_out[s].grow(cst * out_per_stack)))
            return rc;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<int> todo;
    int downloaded = 0;  // chunks whose download has completed
    bool closing = false, failed = false;
    std::thread helper([&] {
        if (hipSetDevice(c->device) != hipSuccess) {
            std::lock_guard<std::mutex> lk(mu);
            failed = true;
        }
        for (;;) {
            int i;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !todo.empty() || closing; });
                if (todo.empty()) return;
                i = todo.front();
                todo.pop_front();
            }
            const int s = i & 1, st0 = i * cst, ns = (st0 + cst <= n_stacks) ? cst : n_stacks - st0;
            bool ok = !failed && hipStreamWaitEvent(c->s_down, c->pe_done[s], 0) == hipSuccess &&
                      hipMemcpyAsync((char*)host_out + (size_t)st0 * out_per_stack, c->p_out[s].p, ns * out_per_stack,
                                     hipMemcpyDeviceToHost, c->s_down) == hipSuccess &&
                      hipStreamSynchronize(c->s_down) == hipSuccess;
            {
                std::lock_guard<std::mutex> lk(mu);
                if (!ok) failed = true;
                downloaded++;
            }
            cv.notify_all();
        }
    });
    for (int i = 0; i < n_chunks && rc == DCT3D_OK; i++) {
        const int s = i & 1, st0 = i * cst, ns = (st0 + cst <= n_stacks) ? cst : n_stacks - st0;
        if (host_in) {  // (no upload when the input is already on the device)
            if (i >= 2 && hipStreamWaitEvent(c->s_up, c->pe_done[s], 0) != hipSuccess) rc = DCT3D_EDEVICE;
            if (!rc && (hipMemcpyAsync(c->p_in[s].p, (const char*)host_in + (size_t)st0 * in_per_stack,
                                       ns * in_per_stack, hipMemcpyHostToDevice, c->s_up) != hipSuccess ||
                        hipEventRecord(c->pe_in[s], c->s_up) != hipSuccess ||
                        hipStreamWaitEvent(c->stream, c->pe_in[s], 0) != hipSuccess))
                rc = DCT3D_EDEVICE;
        }
        {  // slot s's previous download (chunk i - 2) must be finished before its kernels overwrite it
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return downloaded >= i - 1 || failed; });
            if (failed) rc = DCT3D_EDEVICE;
        }
        if (!rc) rc = compute(c->p_in[s].p, c->p_out[s].p, st0, ns);
        if (!rc && hipEventRecord(c->pe_done[s], c->stream) != hipSuccess) rc = DCT3D_EDEVICE;
        if (!rc) {
            std::lock_guard<std::mutex> lk(mu);
            todo.push_back(i);
        }
        cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        closing = true;
    }
    cv.notify_all();
    helper.join();
    if (failed && !rc) rc = DCT3D_EDEVICE;
    if (hipStreamSynchronize(c->stream) != hipSuccess && !rc) rc = DCT3D_EDEVICE;
    return rc;
}

extern "C" {
// ---- host-pointer entry points (synchronous; the reference's blocking transfers) ----------------
int dct3d_encode_stacks(dct3d_ctx* c, const uint8_t* raster, int w, int h, int n_stacks, int32_t* q, double* dct) {
    if (!c || (!raster && n_stacks) || (!q && n_stacks)) return DCT3D_EINVAL;
    uint64_t n_cubes;
    int rc = check_geometry(c, w, h, n_stacks, &n_cubes);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (n_cubes == 0) return DCT3D_OK;
    const size_t in_bytes = n_cubes * c->plan.cs, out_bytes = in_bytes * sizeof(int32_t);
    if (!dct) {  // pipelined
        const size_t px = in_bytes / n_stacks;
        batch_begin(c);  // every chunk counts into one slot: dct3d_get_stats reports the whole call
        rc = run_pipeline(c, n_stacks, px, px * sizeof(int32_t), raster, q,
                          [&](const void* din, void* dout, int, int ns) {
                              return dct3d_encode_stacks_dev(c, (const uint8_t*)din, w, h, ns, (int32_t*)dout, nullptr);
                          });
        batch_end(c);
        return rc;
    }
    if ((rc = c->h_in.grow(in_bytes)) || (rc = c->h_out.grow(out_bytes))) return rc;
    if (hipMemcpyAsync(c->h_in.p, raster, in_bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return DCT3D_EDEVICE;
    if (dct && (rc = c->h_aux.grow(in_bytes * sizeof(double)))) return rc;
    rc = dct3d_encode_stacks_dev(c, (const uint8_t*)c->h_in.p, w, h, n_stacks, (int32_t*)c->h_out.p,
                                 dct ? (double*)c->h_aux.p : nullptr);
    if (rc) return rc;
    if (dct && hipMemcpyAsync(dct, c->h_aux.p, in_bytes * sizeof(double), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        return DCT3D_EDEVICE;
    if (hipMemcpyAsync(q, c->h_out.p, out_bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return DCT3D_EDEVICE;
    return hipStreamSynchronize(c->stream) == hipSuccess ? DCT3D_OK : DCT3D_EDEVICE;
}

int dct3d_decode_stacks(dct3d_ctx* c, const int32_t* q, int w, int h, int n_stacks, uint8_t* raster) {
    if (!c || (!raster && n_stacks) || (!q && n_stacks)) return DCT3D_EINVAL;
    uint64_t n_cubes;
    int rc = check_geometry(c, w, h, n_stacks, &n_cubes);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (n_cubes == 0) return DCT3D_OK;
    const size_t px = n_cubes * c->plan.cs / n_stacks;
    batch_begin(c);
    rc = run_pipeline(c, n_stacks, px * sizeof(int32_t), px, q, raster, [&](const void* din, void* dout, int, int ns) {
        return dct3d_decode_stacks_dev(c, (const int32_t*)din, w, h, ns, (uint8_t*)dout);
    });
    batch_end(c);
    return rc;
}

// ---- drop-in (A): float cube-major <-> float cube-major --------------------------------------
// one launch of the float kernel, timed like the fused kernels when profiling is on (no auxiliary launch:
// the second event pair brackets nothing)
static int cube_f32_dev(dct3d_ctx* c, const float* d_in, size_t n_cubes, float* d_out, bool inverse) {
    if (!c || (n_cubes && (!d_in || !d_out)) || n_cubes >= (1ull << 31) / 8) return DCT3D_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (!n_cubes) return DCT3D_OK;
    hipEvent_t* ev = timing_slot(c);
    if (ev) (void)hipEventRecord(ev[0], c->stream);
    if (launch_cube_f32(c->bd, inverse, d_in, d_out, (uint32_t)n_cubes, c->stream)) return DCT3D_EKERNEL;
    if (ev) {
        (void)hipEventRecord(ev[1], c->stream);
        (void)hipEventRecord(ev[2], c->stream);
        (void)hipEventRecord(ev[3], c->stream);
    }
    c->last_units = n_cubes * (uint64_t)c->plan.cs;
    c->last_valid = false;  // no flag counters for the float path
    c->last_count_slot = -1;
    return DCT3D_OK;
}

int dct3d_forward_f32_dev(dct3d_ctx* c, const float* d_in, size_t n_cubes, float* d_out) {
    return cube_f32_dev(c, d_in, n_cubes, d_out, false);
}

int dct3d_inverse_f32_dev(dct3d_ctx* c, const float* d_in, size_t n_cubes, float* d_out) {
    return cube_f32_dev(c, d_in, n_cubes, d_out, true);
}

static int cube_f32_host(dct3d_ctx* c, const float* in, size_t n_cubes, float* out, bool inverse) {
    if (!c || (n_cubes && (!in || !out)) || n_cubes >= (1ull << 31) / 8) return DCT3D_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (!n_cubes) return DCT3D_OK;
    const size_t bytes = n_cubes * c->plan.cs * sizeof(float);
    int rc;
    if ((rc = c->h_in.grow(bytes)) || (rc = c->h_out.grow(bytes))) return rc;
    if (hipMemcpyAsync(c->h_in.p, in, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return DCT3D_EDEVICE;
    if (launch_cube_f32(c->bd, inverse, (const float*)c->h_in.p, (float*)c->h_out.p, (uint32_t)n_cubes, c->stream))
        return DCT3D_EKERNEL;
    if (hipMemcpyAsync(out, c->h_out.p, bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return DCT3D_EDEVICE;
    return hipStreamSynchronize(c->stream) == hipSuccess ? DCT3D_OK : DCT3D_EDEVICE;
}

int dct3d_forward_f32(dct3d_ctx* c, const float* in, size_t n_cubes, float* out) {
    return cube_f32_host(c, in, n_cubes, out, false);
}

int dct3d_inverse_f32(dct3d_ctx* c, const float* in, size_t n_cubes, float* out) {
    return cube_f32_host(c, in, n_cubes, out, true);
}

// ---- Exp-Golomb stage ----------------------------------------------------------------------------
int dct3d_diagonal_order(int bw, int bh, int bd, uint16_t* out) {
    if (!out || bw != 8 || bh != 8 || (bd != 8 && bd != 4)) return DCT3D_EINVAL;
    diagonal_order(bw, bh, bd, out);
    return DCT3D_OK;
}

static int eg_run(dct3d_ctx* c, const int32_t* d_q, uint64_t n_cubes, uint8_t carry_byte, int carry_bits,
                  uint32_t* d_out, uint64_t out_cap, uint64_t* total_bits) {
    const uint64_t n_chunks = (n_cubes + 4095) / 4096;
    int rc = c->d_eg_bits.grow(n_cubes * sizeof(uint32_t));
    if (!rc) rc = c->d_eg_off.grow(n_cubes * sizeof(uint64_t));
    if (!rc) rc = c->d_eg_bsum.grow((n_chunks + 1) * sizeof(uint64_t));
    if (!rc) rc = c->d_eg_ht.grow(2 * n_cubes * sizeof(uint32_t));
    if (rc) return rc;
    uint64_t* const sw = eg_status_begin(c, &rc);
    if (rc) return rc;
    EgParams P{};
    P.q = d_q;
    P.n_cubes = n_cubes;
    P.diag = (const uint16_t*)c->d_diag.p;
    P.bits = (uint32_t*)c->d_eg_bits.p;
    P.off = (uint64_t*)c->d_eg_off.p;
    P.bsum = (uint64_t*)c->d_eg_bsum.p;
    P.status = sw;
    eg_status_handoff(c, P);  // the stitch kernel (the last of launch_eg_encode) hands the words over
    P.head = (uint32_t*)c->d_eg_ht.p;
    P.tail = (uint32_t*)c->d_eg_ht.p + n_cubes;
    P.out = d_out;
    P.out_cap_words = out_cap / 4;
    P.carry_bits = (uint32_t)carry_bits;
    P.carry_byte = carry_byte;
    if (launch_eg_encode(c->bd, P, c->stream)) return DCT3D_EKERNEL;
    uint64_t st[2] = {0, 0};
    if (eg_status_end(c, true, sw, st, P.seq)) return DCT3D_EDEVICE;
    if (total_bits) *total_bits = st[0];
    if (st[1] & 2) return DCT3D_EINVAL;
    if (st[1] & 1) return DCT3D_ENOSPC;
    return DCT3D_OK;
}

int dct3d_eg_encode_dev(dct3d_ctx* c, const int32_t* d_q, uint64_t n_cubes, uint8_t carry_byte, int carry_bits,
                        uint8_t* d_out, uint64_t out_cap, uint64_t* total_bits) {
    if (!c || carry_bits < 0 || carry_bits > 7 || (n_cubes && (!d_q || !d_out)) || ((uintptr_t)d_out & 3))
        return DCT3D_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (n_cubes == 0) {
        if (total_bits) *total_bits = (uint64_t)carry_bits;
        if (carry_bits == 0) return DCT3D_OK;
        if (out_cap < 4) return DCT3D_ENOSPC;
        const uint32_t w = carry_byte & (0xFF00u >> carry_bits);
        return hipMemcpy(d_out, &w, 4, hipMemcpyHostToDevice) == hipSuccess ? DCT3D_OK : DCT3D_EDEVICE;
    }
    return eg_run(c, d_q, n_cubes, carry_byte, carry_bits, (uint32_t*)d_out, out_cap, total_bits);
}

// Fused device path: encode_eg_kernel (transform, quantise, in-wave exact replay, lane-level
// Exp-Golomb into slots) -> scan over segments -> eg_compact_kernel -> eg_stitch_kernel.
int dct3d_encode_eg_dev(dct3d_ctx* c, const uint8_t* d_raster, int w, int h, int n_stacks, uint8_t carry_byte,
                        int carry_bits, uint8_t* d_out, uint64_t out_cap, uint64_t* total_bits) {
    if (!c || (!d_raster && n_stacks) || carry_bits < 0 || carry_bits > 7 || ((uintptr_t)d_out & 3)) return DCT3D_EINVAL;
    uint64_t n_cubes;
    int rc = check_geometry(c, w, h, n_stacks, &n_cubes);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    c->last_valid = false;
    c->last_count_slot = -1;
    if (n_cubes == 0) return dct3d_eg_encode_dev(c, nullptr, 0, carry_byte, carry_bits, d_out, out_cap, total_bits);
    if (!d_out) return DCT3D_EINVAL;
    const int D = c->bd;
    const uint64_t n_seg = (n_cubes + 7) / 8, n_chunks = (n_seg + 4095) / 4096;
    // worst case per lane: cs/8 values x 27 bits (|q| <= 255 sqrt(cs) -> codes <= 27 bits)
    const uint32_t seg_cap = (uint32_t)(64 * (((c->plan.cs / 8) * 27 + 31) / 32));
    // two passes: K1 codes into per-segment slots, then scan + compaction (a single pass by decoupled
    // look-back wrote the same stream but measured slower: DESIGN.md §4b)
    if ((rc = c->d_egf_slot.grow(n_seg * seg_cap * sizeof(uint32_t))) ||
        (rc = c->d_eg_bits.grow(n_seg * sizeof(uint32_t))) ||
        (rc = c->d_eg_off.grow(n_seg * sizeof(uint64_t))) || (rc = c->d_eg_bsum.grow((n_chunks + 1) * sizeof(uint64_t))) ||
        (rc = c->d_eg_ht.grow(2 * n_seg * sizeof(uint32_t))))
        return rc;
    uint64_t* const sw = eg_status_begin(c, &rc);
    if (rc) return rc;
    const uint64_t plane = (uint64_t)w * h;
    EncodeParams P{};
    P.raster = d_raster;
    P.out = nullptr;
    P.n_cubes = (uint32_t)n_cubes;
    P.g_base = 0;
    P.cubes_per_stack = (uint32_t)((w / 8) * (h / 8));
    P.nbx = (uint32_t)(w / 8);
    set_fast_div(P);
    P.width = (uint32_t)w;
    P.plane = plane;
    P.stack_stride = plane * D;
    P.coef_dc = c->plan.coef_dc;
    const float* tabs = (const float*)c->d_tabs.p;
    P.tab_rstep = tabs;
    P.tab_G = tabs + kMaxS;
    P.tab_E = tabs + 2 * kMaxS;
    EgFusedParams E;
    E.ngroups = (const int32_t*)c->d_ngroups.p;
    E.coef = (const double*)c->d_coef.p;
    E.group_of = (const uint8_t*)c->d_group_of.p;
    E.diag = (const uint16_t*)c->d_diag.p;
    E.slot = (uint32_t*)c->d_egf_slot.p;
    E.seg_cap = seg_cap;
    E.seg_bits = (uint32_t*)c->d_eg_bits.p;
    EgParams G{};
    G.q = nullptr;
    G.n_cubes = n_seg;  // segments
    G.diag = E.diag;
    G.bits = E.seg_bits;
    G.off = (uint64_t*)c->d_eg_off.p;
    G.bsum = (uint64_t*)c->d_eg_bsum.p;
    G.status = sw;
    eg_status_handoff(c, G);  // the stitch kernel (the last of launch_eg_compact) hands the words over
    // (Round 6: handed over by the compaction's block 0 instead, the call returning while the compaction and
    // the stitch ran, the compaction slowed 151 -> 205 us beside the next call's launches: c7 +15-25 us per
    // call, profiles/r06/gaps/async7.  The stream decode's consumer, compute-bound, does not slow.)
    G.head = (uint32_t*)c->d_eg_ht.p;
    G.tail = (uint32_t*)c->d_eg_ht.p + n_seg;
    G.out = (uint32_t*)d_out;
    G.out_cap_words = out_cap / 4;
    G.carry_bits = (uint32_t)carry_bits;
    G.carry_byte = carry_byte;
    uint64_t st[2] = {0, 0};
    hipEvent_t* ev = timing_slot(c);
    if (ev) (void)hipEventRecord(ev[0], c->stream);
    if (launch_encode_eg(D, P, E, c->stream)) return DCT3D_EKERNEL;
    if (ev) (void)hipEventRecord(ev[1], c->stream);
    if (ev) (void)hipEventRecord(ev[2], c->stream);
    if (launch_eg_compact(G, E.slot, seg_cap, c->stream)) return DCT3D_EKERNEL;
    if (ev) (void)hipEventRecord(ev[3], c->stream);
    if (eg_status_end(c, true, sw, st, G.seq)) return DCT3D_EDEVICE;
    if (total_bits) *total_bits = st[0];
    c->last_units = n_cubes * (uint64_t)c->plan.cs;
    if (st[1] & 1) return DCT3D_ENOSPC;
    return DCT3D_OK;
}

int dct3d_encode_eg(dct3d_ctx* c, const uint8_t* raster, int w, int h, int n_stacks, uint8_t carry_byte,
                    int carry_bits, uint64_t* total_bits) {
    if (!c || (!raster && n_stacks) || carry_bits < 0 || carry_bits > 7) return DCT3D_EINVAL;
    uint64_t n_cubes;
    int rc = check_geometry(c, w, h, n_stacks, &n_cubes);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    c->eg_last_bytes = 0;
    const size_t in_bytes = n_cubes * c->plan.cs;
    if ((rc = c->h_in.grow(in_bytes ? in_bytes : 1)) || (rc = c->d_eg_q.grow((in_bytes ? in_bytes : 1) * sizeof(int32_t))))
        return rc;
    if (n_cubes && hipMemcpyAsync(c->h_in.p, raster, in_bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return DCT3D_EDEVICE;
    const bool two_step = c->opt_eg_two_step;  // A/B option: int32 cube-major, then the stand-alone EG stage
    if (!two_step) {
        uint64_t cap = in_bytes + 64, tb = 0;
        for (int attempt = 0; attempt < 2; attempt++) {
            if ((rc = c->d_eg_out.grow(cap))) return rc;
            rc = dct3d_encode_eg_dev(c, (const uint8_t*)c->h_in.p, w, h, n_stacks, carry_byte, carry_bits,
                                     (uint8_t*)c->d_eg_out.p, c->d_eg_out.bytes, &tb);
            if (rc != DCT3D_ENOSPC) break;
            cap = (tb + 31) / 32 * 4 + 64;
        }
        if (rc) return rc;
        if (total_bits) *total_bits = tb;
        c->eg_last_bytes = (tb + 7) / 8;
        return DCT3D_OK;
    }
    if (n_cubes && (rc = dct3d_encode_stacks_dev(c, (const uint8_t*)c->h_in.p, w, h, n_stacks, (int32_t*)c->d_eg_q.p, nullptr)))
        return rc;
    // first try: 1 byte per value (8 bits / value; typical content needs 1.5-4), grown to fit on ENOSPC
    uint64_t cap = in_bytes + 64, tb = 0;
    for (int attempt = 0; attempt < 2; attempt++) {
        if ((rc = c->d_eg_out.grow(cap))) return rc;
        rc = n_cubes ? eg_run(c, (const int32_t*)c->d_eg_q.p, n_cubes, carry_byte, carry_bits, (uint32_t*)c->d_eg_out.p,
                              c->d_eg_out.bytes, &tb)
                     : dct3d_eg_encode_dev(c, nullptr, 0, carry_byte, carry_bits, (uint8_t*)c->d_eg_out.p,
                                           c->d_eg_out.bytes, &tb);
        if (rc != DCT3D_ENOSPC) break;
        cap = (tb + 31) / 32 * 4 + 64;
    }
    if (rc) return rc;
    if (total_bits) *total_bits = tb;
    c->eg_last_bytes = (tb + 7) / 8;
    return DCT3D_OK;
}

int dct3d_eg_fetch(dct3d_ctx* c, uint8_t* out, uint64_t nbytes) {
    if (!c || (nbytes && !out) || nbytes > c->eg_last_bytes) return DCT3D_EINVAL;
    if (nbytes == 0) return DCT3D_OK;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (hipMemcpyAsync(out, c->d_eg_out.p, nbytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return DCT3D_EDEVICE;
    return DCT3D_OK;
}

// Stream decode front: sync passes until the chunk exits converge, the scan of per-chunk code counts,
// the mark pass (bit position of every 32nd value).  No host wait after the last pass; the caller's
// consumer kernel (emit / fused decode) skips itself on a corrupt or short stream, and eg_decode_status
// reports it.  spec (with resolve): no host wait after pass 0 either -- the scan, the mark pass and the
// consumer are enqueued behind it at once; the mark pass reads the pass's verdict (status[0]) first and,
// should a chunk not have resolved (never seen on encoder output), writes no marks and flags status[2]
// bit 4, the consumer skips itself, and eg_decode_status asks the caller to rerun without speculation
// (kEgRetry).  This takes the host round trip between pass 0 and the scan off every call.
constexpr int kEgRetry = 1000;
static int eg_decode_front(dct3d_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, uint64_t start_bit, uint64_t n_cubes,
                           EgDecParams& D, bool spec) {
    const uint64_t limit = nbytes * 8;
    const uint64_t n_chunks = (limit - start_bit + kEgChunkBits - 1) / kEgChunkBits;
    const uint64_t n_scan = (n_chunks + 4095) / 4096;
    int rc = c->d_egd_exit.grow(2 * n_chunks * sizeof(uint64_t));
    if (!rc) rc = c->d_eg_bits.grow(n_chunks * sizeof(uint32_t));
    if (!rc) rc = c->d_eg_off.grow(16 * n_scan * sizeof(uint32_t));  // the scan's parts (launch_eg_dscan)
    if (!rc) rc = c->d_eg_bsum.grow((n_scan + 1) * sizeof(uint64_t));
    const uint64_t n_marks = n_cubes * (uint64_t)c->plan.cs / 32;
    const uint64_t n_mark_groups = n_marks / kMarkGroup + 1;
    if (!rc) rc = c->d_egd_mark.grow(n_mark_groups * sizeof(uint64_t) + (n_marks + 1) * sizeof(uint16_t));
    if (rc) return rc;
    D.words = (const uint32_t*)d_bytes;
    D.n_words = (nbytes + 3) / 4;
    D.start_bit = start_bit;
    D.limit_bit = limit;
    D.n_chunks = n_chunks;
    D.n_values = n_cubes * (uint64_t)c->plan.cs;
    D.cs = c->plan.cs;
    D.diag = (const uint16_t*)c->d_diag.p;
    uint64_t* ex[2] = {(uint64_t*)c->d_egd_exit.p, (uint64_t*)c->d_egd_exit.p + n_chunks};
    D.count = (uint32_t*)c->d_eg_bits.p;
    D.off = nullptr;
    D.part = (uint32_t*)c->d_eg_off.p;
    D.bsum = (uint64_t*)c->d_eg_bsum.p;
    uint64_t* const st = (uint64_t*)c->d_egd_status.p + 6 * c->egd_slot;  // this call's words
    const bool clean = c->egd_clean[c->egd_slot];
    c->egd_clean[c->egd_slot] = false;
    D.status = st;
    D.status_clear = nullptr;
    D.mark_base = (uint64_t*)c->d_egd_mark.p;
    D.mark = (uint16_t*)(D.mark_base + n_mark_groups);
    D.q = nullptr;
    D.status_host = nullptr;
    if (spec && c->opt_eg_fused_front) {
        // A/B option: the fused front, one launch (eg_front_kernel); the consumer reads its verdict on the device
        const uint64_t nb = front_blocks(n_chunks);
        if ((rc = c->d_egd_desc.grow(nb * sizeof(uint64_t)))) return rc;
        if ((!clean && hipMemsetAsync(st, 0, kEgdStatusBytes, c->stream) != hipSuccess) ||
            hipMemsetAsync(c->d_egd_desc.p, 0, nb * sizeof(uint64_t), c->stream) != hipSuccess)
            return DCT3D_EDEVICE;
        if (launch_eg_front(D, (uint64_t*)c->d_egd_desc.p, c->opt_eg_force_retry ? 1 : 0, c->stream)) return DCT3D_EKERNEL;
        return DCT3D_OK;
    }
    // sync passes until no chunk exit changes (pass 0 parses from the nominal chunk starts and, resolving,
    // usually proves every chunk in sync by itself; otherwise confirming passes follow); at most
    // n_chunks + 1 passes by induction from chunk 0.  DCT3D_OPT_EG_NO_RESOLVE: always confirm (A/B, tests)
    const bool resolve = !c->opt_eg_no_resolve;
    int cur = 0;
    for (uint64_t it = 0; it <= n_chunks + 1; it++) {
        if (!(it == 0 && clean) && hipMemsetAsync(st, 0, kEgdStatusBytes, c->stream) != hipSuccess) return DCT3D_EDEVICE;
        D.exit_in = ex[cur];
        D.exit_out = ex[cur ^ 1];
        if (launch_eg_sync(D, (int)(it < 2 ? it : 1), resolve, c->stream)) return DCT3D_EKERNEL;
        cur ^= 1;
        if (it == 0 && !resolve) continue;
        if (it == 0 && spec) {  // speculative front: the verdict is read on the device (eg_mark_kernel)
            if (c->opt_eg_force_retry && hipMemsetAsync(st, 0x01, 1, c->stream) != hipSuccess)
                return DCT3D_EDEVICE;
            break;
        }
        uint64_t changed = 0;
        if (read_status(c, st, 8, &changed)) return DCT3D_EDEVICE;
        if (!changed) break;
        if (it == n_chunks + 1) return DCT3D_EINVAL;  // cannot happen: every pass fixes one more chunk
    }
    // value index of each chunk's first codeword
    EgParams S;
    memset(&S, 0, sizeof(S));
    S.n_cubes = n_chunks;
    S.bits = D.count;
    S.bsum = D.bsum;
    S.status = D.status + 4;  // zeroed with the decode's words
    S.out_cap_words = ~0ull;
    if (launch_eg_dscan(D, S, c->stream)) return DCT3D_EKERNEL;
    D.exit_in = ex[cur];  // the converged exits
    if (launch_eg_mark(D, c->stream)) return DCT3D_EKERNEL;
    return DCT3D_OK;
}

// waits for the stream; the decode's verdict (corrupt: EINVAL, too short: ENODATA) and end bit (the
// consumer wrote the words to the host itself when D.status_host is set)
// The fused decode's verdict is final once the mark pass has run: the consumer's block 0 hands it over as
// the consumer starts (h_status[6] = the call's sequence number, after the words), and the call returns then,
// while the consumer still runs -- the raster completes on the context stream, as every *_dev output does,
// and the caller's next call is queued behind it (round 6: the synchronous return left ~50 us per call with
// the device idle between the consumer's end and the next call's first kernel, profiles/r06/gaps/).
// polls the pinned word h_status[word] for the call's hand-off tag (hand_off_tag: its sequence number in the
// top 16 bits) and returns the tag's value and flags
static int wait_tag(dct3d_ctx* c, int word, uint64_t seq, uint64_t* value, uint32_t* flags) {
    const volatile uint64_t* h = c->h_status;
    uint64_t t = 0;
    for (uint32_t n = 1;; n++) {
        t = h[word];
        if ((t >> 48) == (seq & 0xFFFFu)) break;
        if ((n & 255u) == 0u) {  // now and then: has the stream ended (or failed) without the hand-off?
            const hipError_t e = hipStreamQuery(c->stream);
            if (e != hipSuccess && e != hipErrorNotReady) return DCT3D_EDEVICE;
            if (e == hipSuccess && (h[word] >> 48) != (seq & 0xFFFFu)) return DCT3D_EDEVICE;
        }
        // a long call (a large stream, a busy device): after ~64 k polls the host thread yields its core
        if (n < 65536u) __builtin_ia32_pause();
        else std::this_thread::yield();
    }
    t = h[word];
    *value = t & kTagValueMask;
    *flags = (uint32_t)(t >> 40) & 0xFFu;
    return DCT3D_OK;
}
// the decode's verdict from the tag: w[1] = end bit, w[2] = flags, w[4] = a total that passes the short
// check (the tag's flag 8 says short); the whole words after the stream when the end bit did not fit
static int egd_wait_verdict(dct3d_ctx* c, const EgDecParams& D, uint64_t* w) {
    uint64_t v = 0;
    uint32_t fl = 0;
    if (wait_tag(c, 6, D.seq, &v, &fl)) return DCT3D_EDEVICE;
    if (fl & kTagOverflow) {
        if (stream_wait(c)) return DCT3D_EDEVICE;
        memcpy(w, c->h_status, kEgdStatusBytes);
        return DCT3D_OK;
    }
    w[1] = v;
    w[2] = fl & 7u;
    w[4] = (fl & 8u) ? 0u : D.n_values;
    return DCT3D_OK;
}
static int eg_decode_status(dct3d_ctx* c, const EgDecParams& D, uint64_t* end_bit) {
    uint64_t w[6] = {0, 0, 0, 0, 0, 0};
    if (D.status_host) {
        if (egd_wait_verdict(c, D, w)) return DCT3D_EDEVICE;
    } else if (read_status(c, D.status, kEgdStatusBytes, w)) {
        return DCT3D_EDEVICE;
    }
    c->egd_slot ^= 1;  // the next call's words
    const uint64_t* st = w;         // the decode's words
    const uint64_t* total = w + 4;  // the scan's: total bits, flags
    if (st[2] & 4) return kEgRetry;  // a speculative front whose pass 0 did not resolve: rerun
    if (st[2] & 1) return DCT3D_EINVAL;
    if ((st[2] & 2) || total[0] < D.n_values) return DCT3D_ENODATA;
    if (end_bit) *end_bit = st[1];
    return DCT3D_OK;
}

int dct3d_eg_decode_dev(dct3d_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, uint64_t start_bit, uint64_t n_cubes,
                        int32_t* d_q, uint64_t* end_bit) {
    if (!c || (n_cubes && (!d_bytes || !d_q)) || ((uintptr_t)d_bytes & 3)) return DCT3D_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (end_bit) *end_bit = start_bit;
    if (n_cubes == 0) return DCT3D_OK;
    if (start_bit >= nbytes * 8) return DCT3D_ENODATA;
    for (int spec = 1;; spec = 0) {
        EgDecParams D{};
        int rc = eg_decode_front(c, d_bytes, nbytes, start_bit, n_cubes, D, spec && !c->opt_eg_no_resolve);
        if (rc) return rc;
        D.q = d_q;
        if (launch_eg_emit(c->bd, D, c->stream)) return DCT3D_EKERNEL;
        rc = eg_decode_status(c, D, end_bit);
        if (rc != kEgRetry || !spec) return rc == kEgRetry ? DCT3D_EDEVICE : rc;
    }
}

// Fused stream -> raster decode of stacks [st0, st0 + ns) after eg_decode_front: the decode kernel parses
// its cubes at the marks (no int32 cube-major intermediate) and replays uncertified cubes in the wave by
// re-parsing them.  out_stack0 = where stack st0 goes (the raster pointer is rebased so that the
// kernels' global cube indices land in it).
}  // extern "C"
// A decode_eg_kernel launch starts on a consumer group (kMarkGroup marks = 2,048 values: the group's first
// whole position is in mark_base, and the group's end is the next group's first): its first stack st0 must
// put st0 * cubes-per-stack * cs on a multiple of 2,048 values.  The smallest stack count that does for a
// w x h frame (1 at 1080p; 8 for a frame of an odd number of 8x8x8 cubes).  (Round 6: the host path's
// chunks of stacks started anywhere, and a chunk starting inside a group parsed past its window.)
static int eg_stack_align(const dct3d_ctx* c, int w, int h) {
    const uint64_t per = (uint64_t)(w / c->bw) * (uint64_t)(h / c->bh) * (uint64_t)c->plan.cs;
    const uint64_t grp = kMarkGroup * 32;
    uint64_t a = per % grp, b = grp;  // gcd(per, grp)
    while (a) {
        const uint64_t t = b % a;
        b = a;
        a = t;
    }
    return (int)(grp / b);
}
static int decode_eg_range(dct3d_ctx* c, const EgDecParams& E, int w, int h, int st0, int ns, uint8_t* out_stack0) {
    const int D = c->bd;
    const uint64_t plane = (uint64_t)w * h;
    const uint64_t cps = (uint64_t)(w / 8) * (h / 8);
    uint8_t* out = out_stack0 - (size_t)st0 * plane * D;  // rebased: stack st0 at out_stack0
    DecodeParams P;
    P.in = nullptr;
    P.out = out;
    P.cube_base = (uint32_t)(st0 * cps);
    P.n_cubes = (uint32_t)((st0 + ns) * cps);
    P.cubes_per_stack = (uint32_t)cps;
    P.nbx = (uint32_t)(w / 8);
    set_fast_div(P);
    P.width = (uint32_t)w;
    P.plane = plane;
    P.stack_stride = plane * D;
    P.dec_G = c->plan.dec_G;
    P.dec_E = c->plan.dec_E;
    P.dec_l1_max = c->plan.dec_l1_max;
    P.blk_store = (w / 8) % 2 == 0 && plane * D < (1ull << 32) ? 1u : 0u;  // dec_store_tile's conditions
    P.dec_E += c->opt_dec_margin;  // test option (see above)
    set_dec_replay(c, P);
    hipEvent_t* ev = timing_slot(c);
    if (ev) (void)hipEventRecord(ev[0], c->stream);
    if (launch_decode_eg(D, P, E, c->opt_eg_dec_groups ? c->opt_eg_dec_groups : 8, c->stream)) return DCT3D_EKERNEL;
    if (ev) {
        (void)hipEventRecord(ev[1], c->stream);
        (void)hipEventRecord(ev[2], c->stream);
        (void)hipEventRecord(ev[3], c->stream);
    }
    count_slot_used(c, (uint64_t)ns * cps * (uint64_t)c->plan.cs);
    return DCT3D_OK;
}
extern "C" {

// Fused: device stream -> device raster.  On a corrupt stream the decode kernel skips itself; on a short
// one it decodes whatever the marks hold (bounded windows); the error is returned either way.
int dct3d_decode_eg_dev(dct3d_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, uint64_t start_bit, int w, int h,
                        int n_stacks, uint8_t* d_raster, uint64_t* end_bit) {
    if (!c || (n_stacks && (!d_bytes || !d_raster)) || ((uintptr_t)d_bytes & 3)) return DCT3D_EINVAL;
    uint64_t n_cubes;
    int rc = check_geometry(c, w, h, n_stacks, &n_cubes);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    c->last_valid = false;
    c->last_count_slot = -1;
    if (end_bit) *end_bit = start_bit;
    if (n_cubes == 0) return DCT3D_OK;
    if (start_bit >= nbytes * 8) return DCT3D_ENODATA;
    for (int spec = 1;; spec = 0) {
        EgDecParams E{};
        if ((rc = eg_decode_front(c, d_bytes, nbytes, start_bit, n_cubes, E, spec && !c->opt_eg_no_resolve))) return rc;
        E.status_host = c->h_status_dev;  // the consumer hands the verdict to the host (nullptr: a copy)
        E.seq = ++c->egd_seq;
        E.status_clear = (uint64_t*)c->d_egd_status.p + 6 * (c->egd_slot ^ 1);  // and zeroes the next call's
        if ((rc = decode_eg_range(c, E, w, h, 0, n_stacks, d_raster))) return rc;
        c->egd_clean[c->egd_slot ^ 1] = true;
        rc = eg_decode_status(c, E, end_bit);
        if (rc != kEgRetry || !spec) return rc == kEgRetry ? DCT3D_EDEVICE : rc;
    }
}

int dct3d_decode_eg(dct3d_ctx* c, const uint8_t* bytes, uint64_t nbytes, int start_bit, int w, int h, int n_stacks,
                    uint8_t* raster, uint64_t* end_bit) {
    if (!c || (n_stacks && (!bytes || !raster)) || start_bit < 0 || start_bit > 7) return DCT3D_EINVAL;
    uint64_t n_cubes;
    int rc = check_geometry(c, w, h, n_stacks, &n_cubes);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return DCT3D_EDEVICE;
    if (end_bit) *end_bit = (uint64_t)start_bit;
    if (n_cubes == 0) return DCT3D_OK;
    if ((uint64_t)start_bit >= nbytes * 8) return DCT3D_ENODATA;
    if ((rc = c->d_egd_in.grow((nbytes + 8) & ~(uint64_t)3))) return rc;
    if (hipMemcpyAsync(c->d_egd_in.p, bytes, nbytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return DCT3D_EDEVICE;
    for (int spec = 1;; spec = 0) {
        EgDecParams E{};
        if ((rc = eg_decode_front(c, (const uint8_t*)c->d_egd_in.p, nbytes, (uint64_t)start_bit, n_cubes, E,
                                  spec && !c->opt_eg_no_resolve)))
            return rc;
        // the raster leaves in chunks of stacks while the next chunk decodes (the stream is small: no upload)
        const size_t px = n_cubes * c->plan.cs / n_stacks;
        batch_begin(c);
        rc = run_pipeline(c, n_stacks, 0, px, nullptr, raster, [&](const void*, void* dout, int st0, int ns) {
            return decode_eg_range(c, E, w, h, st0, ns, (uint8_t*)dout);
        }, eg_stack_align(c, w, h));  // each chunk's first cube on a consumer group
        batch_end(c);
        if (rc) return rc;
        rc = eg_decode_status(c, E, end_bit);
        if (rc != kEgRetry || !spec) return rc == kEgRetry ? DCT3D_EDEVICE : rc;
    }
}

}  // extern "C"
