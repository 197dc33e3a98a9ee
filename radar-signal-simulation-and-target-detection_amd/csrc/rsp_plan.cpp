// rsp_plan.cpp -- host runtime of librsp: plan construction (geometry analysis of the
// reference's precomputed_data), the C-ABI of include/rsp.h, the device-resident frame
// queue, and the host stages S10/S11 (two-level BFS clustering, fsf:302-407).
#include "rsp.h"
#include "rsp_internal.h"

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

// Error sink and host-only stages live in rsp_host.cpp (plain C++, built and sanitized
// without HIP); these are their hidden entry points.
__attribute__((visibility("hidden"))) int rsp_set_error(int code, const char* fmt, ...);
__attribute__((visibility("hidden"))) void rsp_cluster_frame(const rsp_cluster_params& cp, std::vector<rsp_detection>& dets,
                                                             std::vector<rsp_target>& final_targets);

namespace {

template <class... A>
int fail(int code, const char* fmt, A... a) { return rsp_set_error(code, fmt, a...); }

}  // namespace

namespace {

#define HIPCHK(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(RSP_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                                    \
    } while (0)

using cd = std::complex<double>;

bool is_pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }
int ilog2i(int x) { int l = 0; while ((1 << l) < x) ++l; return l; }

// In-place double FFT (sign -1 forward, +1 inverse, unscaled); O(n^2) DFT if n is not 2^k.
void fft_d(std::vector<cd>& a, int sign) {
    const int n = (int)a.size();
    if (!is_pow2(n)) {
        std::vector<cd> o(n);
        for (int k = 0; k < n; ++k) {
            cd s = 0;
            for (int t = 0; t < n; ++t) s += a[t] * std::polar(1.0, sign * 2.0 * M_PI * ((double)((int64_t)t * k % n)) / n);
            o[k] = s;
        }
        a.swap(o);
        return;
    }
    for (int i = 1, j = 0; i < n; ++i) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    for (int len = 2; len <= n; len <<= 1) {
        for (int i = 0; i < n; i += len) {
            for (int k = 0; k < len / 2; ++k) {
                const cd w = std::polar(1.0, sign * 2.0 * M_PI * k / len);
                const cd u = a[i + k], v = a[i + k + len / 2] * w;
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
        }
    }
}

// Row stride (complex elements, P..P+15) of the factored slow-time DFT's LDS tile: the one whose
// pass-2 reads (k1_dft_rq: lane = subsequence (column, k2) of the first 64, element n + Q k2 of
// its column, and its mirror Q - n + Q k2) take the fewest ds_read_b128 cycles by the gfx950
// bank model (MI355X_MICROARCH.md LDS table: four 16-lane groups, 64 banks of 4 B; identical
// addresses broadcast).  Smallest stride on ties.  The reference frame (R = 4, Q = 83, B = 13):
// stride 332 = P itself is conflict-free.
int rq_pick_stride(int R, int Q, int ncols) {
    static const int grp_first[4][3][2] = {{{0, 4}, {12, 16}, {20, 28}}, {{4, 12}, {16, 20}, {28, 32}},
                                           {{32, 36}, {44, 48}, {52, 60}}, {{36, 44}, {48, 52}, {60, 64}}};
    const int P = R * Q, NS = std::min(ncols * R, 64), Qh = (Q - 1) / 2;
    int best = P, best_cost = INT32_MAX;
    for (int rs = P; rs < P + 16; ++rs) {
        long cost = 0;
        for (int n = 1; n <= Qh; ++n)
            for (int mirror = 0; mirror < 2; ++mirror)
                for (auto& grp : grp_first) {
                    int addr[16], na = 0;   // distinct 16-B addresses of the group's lanes
                    for (auto& rg : grp)
                        for (int l = rg[0]; l < rg[1]; ++l) {
                            if (l >= NS) continue;
                            const int c = l / R, k2 = l % R;
                            const int a = c * rs + Q * k2 + (mirror ? Q - n : n);
                            bool seen = false;   // a broadcast of the same address is free
                            for (int j = 0; j < na; ++j) seen = seen || addr[j] == a;
                            if (!seen) addr[na++] = a;
                        }
                    int cnt[16] = {0}, worst = 1;   // a 16-B slot covers 4 banks: slot a & 15
                    for (int j = 0; j < na; ++j) worst = std::max(worst, ++cnt[addr[j] & 15]);
                    cost += worst;
                }
        if (cost < best_cost) {
            best_cost = (int)cost;
            best = rs;
        }
    }
    return best;
}

// exp(-2 pi i e / n) with e reduced mod n and the angle formed in long double
cd root_of_unity(long long e, long long n) {
    e %= n;
    if (e < 0) e += n;
    const long double a = -2.0L * 3.141592653589793238462643383279502884L * (long double)e / (long double)n;
    return cd((double)std::cos(a), (double)std::sin(a));
}

// Radix sequence for a 2^m-point Stockham FFT: radix 16 passes, remainder as 8/4
// (never a lone radix-2 pass unless m == 1).  pal: a 3-pass plan with the remainder in the
// middle (the overlap-save blocks, rad_bits_pal in rsp_kernels.hip).
void radix_plan(int m, int* nrad, int* rad, bool pal = false) {
    *nrad = 0;
    while (m > 0) {
        const int p = (m == 5) ? 3 : (m >= 4 ? 4 : m);
        rad[(*nrad)++] = 1 << p;
        m -= p;
    }
    if (pal && *nrad == 3) std::swap(rad[1], rad[2]);
}

void push_pass_twiddles(std::vector<cd>& out, int Ns, int R, bool cmp) {
    if (cmp) {
        for (int r = 1; r < R; r *= 2)
            for (int k = 0; k < Ns; ++k) out.push_back(root_of_unity((long long)k * r, (long long)Ns * R));
    } else {
        for (int k = 0; k < Ns; ++k)
            for (int r = 1; r < R; ++r) out.push_back(root_of_unity((long long)k * r, (long long)Ns * R));
    }
}

// Per-pass Stockham twiddle tables of a 2^m-point FFT (radix order reversed if rev),
// concatenated: pass q >= 1 owns Ns_q x (R_q - 1) entries T[k][r-1] = exp(-2 pi i k r / (Ns_q R_q))
// (must match tw_pass_off() in rsp_kernels.hip).  Compact tables (cmp): r = 1, 2, 4, 8 only,
// stored column-major, [i][k] = T[k][2^i] (load_tw in rsp_kernels.hip).
// The angle's numerator is reduced modulo the period first, so every entry is the correctly
// rounded double of the exact root of unity's angle.
void build_pass_twiddles(int m, std::vector<cd>& out, bool rev = false, bool cmp = false, bool pal = false) {
    int nrad, rad[8];
    radix_plan(m, &nrad, rad, pal);
    if (rev) std::reverse(rad, rad + nrad);
    int Ns = 1;
    for (int q = 0; q < nrad; ++q) {
        const int R = rad[q];
        if (q > 0) push_pass_twiddles(out, Ns, R, cmp);
        Ns *= R;
    }
}

// Mixed-radix overlap-save block M = 16 x R1 x 16 (k2_fft_job_mix): a palindrome, so the
// inverse table (reversed radices) is the forward one and only the forward table is stored.
void build_mix_twiddles(int R0, int R1, std::vector<cd>& out, bool cmp) {
    const int rad[3] = {R0, R1, R0};
    int Ns = 1;
    for (int q = 0; q < 3; ++q) {
        const int R = rad[q];
        if (q > 0) push_pass_twiddles(out, Ns, R, cmp);
        Ns *= R;
    }
}

double mround(double x) { return x < 0 ? -std::floor(-x + 0.5) : std::floor(x + 0.5); }

struct Lane {
    hipStream_t stream = nullptr;   // the lane's stream: its batches' kernels and detection read-back
    hipEvent_t tev[4] = {};         // live stage timing: before K1, after K1, K2, K3
    bool timed = false;
    hipEvent_t done = nullptr;
    void* z = nullptr;          // F frames
    void* rdm = nullptr;        // ONE frame: the synchronous paths' RDM (queue frames write the caller's maps)
    void* mag = nullptr;        // F frames
    DevDet* dets = nullptr;     // F x (1 + dcap): record 0 of each frame holds its count
    int dcap = 0;               // device detection-list capacity per frame (grows on demand)
    DevDet* h_dets = nullptr;   // mapped pinned F x (1 + hcap), same layout, written by k_dets_to_host
    DevDet* h_dets_dev = nullptr;
    int hcap = 0;               // host read-back capacity per frame (grows on demand)
    FramePtrs fp{};             // the batch in flight (K3 runs again after a device-list growth)
    int nf = 0;
    int frame_ids[RSP_MAX_F];
    bool busy = false;
};

// Host worker threads for S10/S11 (fsf:302-407) of the queue's frames: a harvested batch's
// frames are clustered in parallel while the host thread goes on launching batches, so the
// clustering neither delays the next launch nor serialises the end of a run (one x2 frame with
// ~250 detections takes ~60 us; eight in a row were ~0.5 ms of host time per batch).
class ClusterPool {
public:
    explicit ClusterPool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~ClusterPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(m_);
            q_.push_back(std::move(f));
            ++pending_;
        }
        cv_.notify_one();
    }
    void wait() {   // every submitted task has finished
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return pending_ == 0; });
    }

private:
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
            std::lock_guard<std::mutex> g(m_);
            if (--pending_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::deque<std::function<void()>> q_;
    int pending_ = 0;
    bool stop_ = false;
};

struct FrameResult {
    int frame_idx;
    int n_dets;
    std::vector<rsp_target> targets;
};

}  // namespace

struct rsp_plan {
    int device = 0;
    Geometry g{};
    DevConsts k{};
    rsp_cluster_params cl{};
    double deltaR = 0, deltaV = 0;
    double p_signal_unscaled = 0, c = 0, fs = 0, wavelength = 0, d = 0, prt = 0;
    int F = 1;
    int det_bound = 1;   // cells under test per frame: the most detections a frame can have
    size_t esz = 16;   // bytes of one complex element (16: complex128, 8: complex64)
    size_t rsz = 8;    // bytes of one real element
    size_t z_elems = 0, rdm_elems = 0, mag_elems = 0;
    std::vector<SegDesc> segs;
    std::vector<K2Job> jobs;
    std::vector<void*> dev_allocs;
    double* d_tx = nullptr;
    double* d_stab = nullptr;     // S4 phasor tables: RSP_MAX_SYNTH_TARGETS x (P + C) complex
    void* d_cube = nullptr;       // staging cube for the synchronous paths
    void* d_aux = nullptr;        // second map for the stage-2 path
    void* d_smap = nullptr;       // rdm_for_cfar_all of the synchronous path (allocated on first request)
    unsigned char* h_stage = nullptr;   // pinned staging for uploads
    size_t h_stage_bytes = 0;
    Lane lanes[RSP_LANES];
    int nlanes = RSP_NLANES;   // lanes (streams) of the throughput queue
    int next_lane = 0;
    // live stage timing of the queue (rsp_set_stage_timing): HIP events around K1/K2/K3 of
    // every batch, summed at harvest
    bool time_stages = false;
    double stage_ms[3] = {0, 0, 0};
    int64_t stage_launches = 0, stage_frames = 0;
    // pending batch of the queue
    const void* pend_in[RSP_MAX_F];
    void* pend_rdm[RSP_MAX_F];  // caller's device RD map of each pending frame (nullptr: kept on chip)
    int pend_ids[RSP_MAX_F];
    int pend_slot[RSP_MAX_F];   // producer-ring slot of each pending frame, -1 = caller's device cube
    int npend = 0;
    // producer ring of the queue (rsp_enqueue_host, rsp_process_targets_multi): device cubes
    // written on up_stream.  slot_ready[s] orders K1 after the write; slot_free[s], recorded after
    // the K1 that read slot s, orders the next write after it.  (nlanes + 1) x F slots: a slot
    // comes round again only after its frame's batch has been launched.
    hipStream_t up_stream = nullptr;
    std::vector<void*> ring;
    std::vector<hipEvent_t> slot_ready, slot_free;
    std::vector<char> slot_used;
    int ring_next = 0;
    std::deque<FrameResult> results;   // deque: push_back keeps the elements the pool writes in place
    std::vector<rsp_detection> last_dets;   // detections of the last synchronous frame (rsp_last_detections)
    std::vector<rsp_target> last_targets;   // its final targets (rsp_last_targets)
    // clustering workers of the queue (created with the first batch of F > 1 frames); every
    // reader of `results` calls results_ready() first.  Declared after `results`: destroyed first.
    std::unique_ptr<ClusterPool> pool;
    void results_ready() const {
        if (pool) pool->wait();
    }

    ~rsp_plan();
    int dalloc_bytes(void** p, size_t bytes) {
        void* q = nullptr;
        if (hipMalloc(&q, bytes + 16) != hipSuccess) return fail(RSP_ERR_NOMEM, "hipMalloc(%zu bytes) failed", bytes);
        dev_allocs.push_back(q);
        *p = q;
        return RSP_OK;
    }
    template <class T>
    int dalloc(T** p, size_t n) {
        void* q = nullptr;
        int rc = dalloc_bytes(&q, n * sizeof(T));
        *p = (T*)q;
        return rc;
    }
    template <class T>
    int upload(T** p, const std::vector<T>& h) {
        int rc = dalloc(p, std::max<size_t>(h.size(), 1));
        if (rc) return rc;
        if (!h.empty()) HIPCHK(hipMemcpy(*p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
        return RSP_OK;
    }
    // complex / real tables in the plan's precision
    int upload_c(const void** p, const std::vector<cd>& h) {
        if (g.prec == RSP_PREC_F64) {
            double* q;
            std::vector<double> v(2 * h.size());
            for (size_t i = 0; i < h.size(); ++i) { v[2 * i] = h[i].real(); v[2 * i + 1] = h[i].imag(); }
            int rc = upload(&q, v);
            *p = q;
            return rc;
        }
        float* q;
        std::vector<float> v(2 * h.size());
        for (size_t i = 0; i < h.size(); ++i) { v[2 * i] = (float)h[i].real(); v[2 * i + 1] = (float)h[i].imag(); }
        int rc = upload(&q, v);
        *p = q;
        return rc;
    }
    int upload_r(const void** p, const std::vector<double>& h) {
        if (g.prec == RSP_PREC_F64) {
            double* q;
            int rc = upload(&q, h);
            *p = q;
            return rc;
        }
        float* q;
        std::vector<float> v(h.begin(), h.end());
        int rc = upload(&q, v);
        *p = q;
        return rc;
    }
};

rsp_plan::~rsp_plan() {
    results_ready();
    (void)hipSetDevice(device);
    for (auto& L : lanes) {
        if (L.stream) (void)hipStreamSynchronize(L.stream);
        if (L.h_dets) (void)hipHostFree(L.h_dets);
        if (L.dets) (void)hipFree(L.dets);
        if (L.done) (void)hipEventDestroy(L.done);
        for (auto& e : L.tev)
            if (e) (void)hipEventDestroy(e);
        if (L.stream) (void)hipStreamDestroy(L.stream);
    }
    if (up_stream) (void)hipStreamSynchronize(up_stream);
    for (auto e : slot_ready) if (e) (void)hipEventDestroy(e);
    for (auto e : slot_free) if (e) (void)hipEventDestroy(e);
    if (up_stream) (void)hipStreamDestroy(up_stream);
    if (h_stage) (void)hipHostFree(h_stage);
    for (void* p : dev_allocs) (void)hipFree(p);
}

namespace {

// ---- geometry analysis ------------------------------------------------------------------
struct Interval { int lo, hi; };

int build_fft_segment(SegDesc& s, const double* mf_fft, int Nfft, int N, int ga, int gb, int seg_lo,
                      std::vector<cd>& H, std::vector<cd>& twM, std::vector<int>& tw_sizes, std::vector<int>& tw_offs,
                      const char* name) {
    std::vector<cd> h(Nfft);
    for (int i = 0; i < Nfft; ++i) h[i] = cd(mf_fft[2 * i], mf_fft[2 * i + 1]);
    fft_d(h, +1);
    double hmax = 0;
    for (auto& v : h) { v /= (double)Nfft; hmax = std::max(hmax, std::abs(v)); }
    if (hmax == 0) return fail(RSP_ERR_INVALID, "%s matched filter is all zero", name);
    int Lh = 0;
    for (int i = 0; i < Nfft; ++i) if (std::abs(h[i]) > 1e-10 * hmax) Lh = i + 1;
    if (gb > Nfft)
        return fail(RSP_ERR_INVALID, "%s gates end at %d beyond N_fft %d (fsf:124-125 index out of range)", name, gb, Nfft);
    const int Ls = std::min(N - seg_lo, Nfft);   // fft(seg, Nfft) truncates or pads
    if (ga < Lh - 1 && Ls + (Lh - 1 - ga) > Nfft)
        return fail(RSP_ERR_UNSUPPORTED, "%s segment: circular aliasing reaches kept gates (L_s=%d L_h=%d N_fft=%d)", name, Ls, Lh, Nfft);
    s.type = 1;
    s.ga = ga; s.gb = gb; s.seg_lo = seg_lo;
    s.Lh = Lh;
    s.lo = std::max(seg_lo, seg_lo + ga - (Lh - 1));
    s.hi = std::min(seg_lo + Ls - 1, seg_lo + gb - 1);
    // overlap-save block size M = 2^k <= 2048 (so that a workgroup owns >= 2 adjacent rows:
    // 128 B contiguous loads of z), the mixed-radix 2560 = 16 x 10 x 16 (one row per workgroup)
    // or 4096 = 16 x 16 x 16 (one row per 4096-point workgroup: x4's 5 956-gate long segment in
    // 2 blocks instead of 5 x 2048); cost model blocks * M * (log2 M + 2)
    const int nout = gb - ga;
    double best = 1e300;
    int bestM = 0;
    const int cand[] = {64, 128, 256, 512, 1024, 2048, 2560, 4096};
    for (int M : cand) {
        const int V = M - Lh + 1;
        if (V < 1) continue;
        const int nb = (nout + V - 1) / V;
        const double cost = (double)nb * M * (std::log2((double)M) + 2);
        if (cost < best * 0.999) { best = cost; bestM = M; }
    }
    if (!bestM) return fail(RSP_ERR_UNSUPPORTED, "%s filter length %d exceeds the 2048-point block", name, Lh);
    const int M = bestM;
    const bool mix = !is_pow2(M);
    s.M = M; s.logM = mix ? 0 : ilog2i(M); s.V = M - Lh + 1;
    s.nblocks = (nout + s.V - 1) / s.V;
    // spectrum of h zero-padded to M, natural order, 1/M folded in
    std::vector<cd> hm(M, 0.0);
    for (int i = 0; i < Lh; ++i) hm[i] = h[i];
    fft_d(hm, -1);
    s.H_off = (int)H.size();
    for (auto& v : hm) H.push_back(v / (double)M);
    int ti = -1;
    for (size_t q = 0; q < tw_sizes.size(); ++q) if (tw_sizes[q] == M) ti = (int)q;
    if (ti < 0) {
        tw_sizes.push_back(M);
        tw_offs.push_back((int)twM.size());
        if (mix) {
            build_mix_twiddles(16, M / 256, twM, true);
        } else {
            build_pass_twiddles(s.logM, twM, false, true, true);   // forward FFT (compact rows, palindromic plan)
            build_pass_twiddles(s.logM, twM, true, true, true);    // inverse FFT (reversed radices)
        }
        ti = (int)tw_sizes.size() - 1;
    }
    s.tw_off = tw_offs[ti];
    return RSP_OK;
}

// Device detection lists of a lane: F x (1 + cap) records (record 0 of a frame = its count).
// The new lists are allocated first and swapped in only on success: a failed growth leaves the
// lane with its old lists and capacity (still consistent for the next launch).
int lane_dets_alloc(rsp_plan* p, Lane& L, int cap) {
    const int ncap = std::max(cap, 1);
    DevDet* nd = nullptr;
    if (hipMalloc((void**)&nd, sizeof(DevDet) * (size_t)(ncap + 1) * p->F) != hipSuccess)
        return fail(RSP_ERR_NOMEM, "hipMalloc of %d-detection lists failed", ncap);
    if (L.dets) HIPCHK(hipFree(L.dets));
    L.dets = nd;
    L.dcap = ncap;
    return RSP_OK;
}

// Mapped, coherent pinned read-back lists of a lane: F x (1 + cap) records, written by
// k_dets_to_host over PCIe after K3 (only the records that exist).
int lane_host_alloc(rsp_plan* p, Lane& L, int cap) {
    if (L.h_dets) HIPCHK(hipHostFree(L.h_dets));
    L.h_dets = L.h_dets_dev = nullptr;
    L.hcap = std::max(cap, 1);
    if (hipHostMalloc((void**)&L.h_dets, sizeof(DevDet) * (size_t)(L.hcap + 1) * p->F,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return fail(RSP_ERR_NOMEM, "pinned %d-detection read-back lists failed", L.hcap);
    HIPCHK(hipHostGetDevicePointer((void**)&L.h_dets_dev, L.h_dets, 0));
    return RSP_OK;
}

int pow2_at_least(int x) {
    int c = 1;
    while (c < x && c < (1 << 30)) c <<= 1;
    return c;
}

int setup_lane(rsp_plan* p, Lane& L) {
    HIPCHK(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&L.done, hipEventDisableTiming));
    for (auto& e : L.tev) HIPCHK(hipEventCreate(&e));
    int rc;
    if ((rc = p->dalloc_bytes(&L.z, p->z_elems * p->F * p->esz))) return rc;
    // one frame (sync paths); F frames when S9 reads the complex map (RSP_PLAN_MONOPULSE_COMPLEX)
    if ((rc = p->dalloc_bytes(&L.rdm, p->rdm_elems * p->esz * (p->g.mono_c ? p->F : 1)))) return rc;
    if ((rc = p->dalloc_bytes(&L.mag, p->mag_elems * p->F * p->rsz))) return rc;
    if ((rc = lane_dets_alloc(p, L, std::min(p->det_bound, 4096)))) return rc;
    return lane_host_alloc(p, L, std::min(p->det_bound, 1024));
}

// rdm[f] = nullptr: K2 keeps frame f's complex RD map on chip and stores only its magnitudes,
// the one input of K3 and S9.  fun_process_single_frame returns final_targets (fsf:13); its
// rdm_13beam is an intermediate, so the throughput queue does not write it to HBM (-10% k2_pc)
// unless the caller hands a map for the frame (rsp_enqueue_device_rdm).  rdm == nullptr: no
// frame writes its map.  The synchronous paths (rsp_process_* with out->rdm, process_stage2)
// run one frame into the lane's own map L.rdm.  With RSP_PLAN_MONOPULSE_COMPLEX K3's S9 reads
// the complex map, so every frame writes one: the caller's, or the lane's own (F frames).
FramePtrs lane_ptrs(const rsp_plan* p, const Lane& L, const void* const* in, int nf, void* const* rdm) {
    FramePtrs fp{};
    for (int f = 0; f < nf; ++f) {
        fp.in[f] = in[f];
        fp.z[f] = (char*)L.z + p->z_elems * p->esz * f;
        fp.rdm[f] = rdm && rdm[f] ? rdm[f] : (p->g.mono_c ? (char*)L.rdm + p->rdm_elems * p->esz * f : nullptr);
        fp.mag[f] = (char*)L.mag + p->mag_elems * p->rsz * f;
        DevDet* rec = L.dets + (size_t)(L.dcap + 1) * f;
        fp.count[f] = reinterpret_cast<int*>(rec);   // zeroed by K1, bumped by K3
        fp.dets[f] = rec + 1;
    }
    return fp;
}

// Enqueue K1 -> K2 -> K3 for nf frames on lane L, plus the async detection read-back.
// smap (optional, one frame): K3 also writes rdm_for_cfar_all there.
#define RSP_K3_TILE_KB 48   // KB of S per K3 tile (48: 2 Doppler bands at P = 128, 3 workgroups per CU)
#define RSP_K3_RT_C128 32   // K3 tile width in range cells, complex double
// A lane's buffers are reused only after harvest has waited for the lane's previous batch.
int launch_batch(rsp_plan* p, Lane& L, const void* const* in, const int* ids, int nf, void* smap = nullptr,
                 const int* slots = nullptr, void* const* rdm = nullptr) {
    FramePtrs fp = lane_ptrs(p, L, in, nf, rdm);
    fp.smap[0] = smap;
    if (slots)   // producer-ring frames: K1 after their upload / synthesis
        for (int f = 0; f < nf; ++f)
            if (slots[f] >= 0) HIPCHK(hipStreamWaitEvent(L.stream, p->slot_ready[slots[f]], 0));
    L.timed = p->time_stages;
    if (L.timed) HIPCHK(hipEventRecord(L.tev[0], L.stream));
    HIPCHK(launch_k1(p->g, p->k, fp, nf, 3, L.stream));
    if (slots)   // K1 has read the cubes: their slots may be written again
        for (int f = 0; f < nf; ++f)
            if (slots[f] >= 0) HIPCHK(hipEventRecord(p->slot_free[slots[f]], L.stream));
    if (L.timed) HIPCHK(hipEventRecord(L.tev[1], L.stream));
    HIPCHK(launch_k2(p->g, p->k, fp, nf, p->g.B * p->g.P, L.stream));
    if (L.timed) HIPCHK(hipEventRecord(L.tev[2], L.stream));
    Geometry g3 = p->g;
    g3.max_dets = L.dcap;
    HIPCHK(launch_k3(g3, p->k, fp, nf, L.stream));
    if (L.timed) HIPCHK(hipEventRecord(L.tev[3], L.stream));
    // every frame's count and detections into the lane's mapped pinned lists (only what exists)
    HIPCHK(launch_dets_to_host(L.dets, L.dcap, L.h_dets_dev, L.hcap, nf, L.stream));
    HIPCHK(hipEventRecord(L.done, L.stream));
    L.fp = fp;
    L.nf = nf;
    for (int f = 0; f < nf; ++f) L.frame_ids[f] = ids[f];
    L.busy = true;
    return RSP_OK;
}

// Wait for lane L, gather its detections and cluster.  The lists have no fixed capacity, like
// all_raw_detections(end+1, :) (fsf:215-221): a frame with more detections than the lane's device
// list grows the list and runs K3 again on the batch (its magnitude maps are still in the lane),
// and a frame with more than the host read-back holds is copied directly once and the read-back
// grown, so that later batches come back whole through k_dets_to_host.
int harvest(rsp_plan* p, Lane& L, std::vector<std::vector<rsp_detection>>* keep_dets = nullptr) {
    if (!L.busy) return RSP_OK;
    HIPCHK(hipEventSynchronize(L.done));
    L.busy = false;
    if (L.timed) {
        for (int i = 0; i < 3; ++i) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, L.tev[i], L.tev[i + 1]));
            p->stage_ms[i] += ms;
        }
        p->stage_launches += 1;
        p->stage_frames += L.nf;
    }
    int cnt[RSP_MAX_F], maxc = 0, rc;
    for (int f = 0; f < L.nf; ++f) {
        cnt[f] = *reinterpret_cast<const int*>(L.h_dets + (size_t)f * (L.hcap + 1));
        maxc = std::max(maxc, cnt[f]);
    }
    const bool regrow = maxc > L.dcap;
    if (regrow) {   // rare: grow the device lists, run K3 again with them, read back directly
        if ((rc = lane_dets_alloc(p, L, std::min(p->det_bound, pow2_at_least(maxc))))) return rc;
        FramePtrs fp = L.fp;
        for (int f = 0; f < L.nf; ++f) {
            DevDet* rec = L.dets + (size_t)(L.dcap + 1) * f;
            fp.count[f] = reinterpret_cast<int*>(rec);
            fp.dets[f] = rec + 1;
        }
        HIPCHK(hipMemset2DAsync(L.dets, sizeof(DevDet) * (L.dcap + 1), 0, sizeof(int), L.nf, L.stream));
        Geometry g3 = p->g;
        g3.max_dets = L.dcap;
        HIPCHK(launch_k3(g3, p->k, fp, L.nf, L.stream));
        HIPCHK(hipStreamSynchronize(L.stream));
        L.fp = fp;
    }
    if (keep_dets) keep_dets->assign(L.nf, {});
    for (int f = 0; f < L.nf; ++f) {
        const DevDet* hrec = L.h_dets + (size_t)f * (L.hcap + 1);
        const DevDet* drec = L.dets + (size_t)(L.dcap + 1) * f;
        FrameResult fr;
        fr.frame_idx = L.frame_ids[f];
        const int n = cnt[f];
        fr.n_dets = n;
        std::vector<rsp_detection> dets(n);
        static_assert(sizeof(DevDet) == sizeof(rsp_detection), "layout");
        const int na = regrow ? 0 : std::min(n, L.hcap);   // already in host memory
        if (na) memcpy(dets.data(), hrec + 1, sizeof(DevDet) * na);
        if (n > na) HIPCHK(hipMemcpy(dets.data() + na, drec + 1 + na, sizeof(DevDet) * (n - na), hipMemcpyDeviceToHost));
        if (keep_dets || L.nf == 1) {   // synchronous frame paths: cluster here
            rsp_cluster_frame(p->cl, dets, fr.targets);
            if (keep_dets) (*keep_dets)[f] = dets;
            p->results.push_back(std::move(fr));
        } else {
            if (!p->pool) p->pool.reset(new ClusterPool(std::max(1, std::min<int>(p->F, 8))));
            p->results.push_back(std::move(fr));
            FrameResult* slot = &p->results.back();
            const rsp_cluster_params cl = p->cl;
            p->pool->submit([cl, slot, d = std::move(dets)]() mutable { rsp_cluster_frame(cl, d, slot->targets); });
        }
    }
    if (maxc > L.hcap && (rc = lane_host_alloc(p, L, std::min(p->det_bound, pow2_at_least(maxc))))) return rc;
    return RSP_OK;
}

int flush_pending(rsp_plan* p) {
    if (!p->npend) return RSP_OK;
    Lane& L = p->lanes[p->next_lane];
    int rc = harvest(p, L);
    if (rc) return rc;
    rc = launch_batch(p, L, p->pend_in, p->pend_ids, p->npend, nullptr, p->pend_slot, p->pend_rdm);
    p->npend = 0;
    p->next_lane = (p->next_lane + 1) % p->nlanes;
    return rc;
}

int drain_all(rsp_plan* p) {
    int rc = flush_pending(p);
    if (rc) return rc;
    // harvest in launch order: the lane launched first is next_lane
    for (int q = 0; q < p->nlanes; ++q) {
        rc = harvest(p, p->lanes[(p->next_lane + q) % p->nlanes]);
        if (rc) return rc;
    }
    p->results_ready();
    return RSP_OK;
}

// Next slot of the producer ring (allocated on first use); up_stream waits until the K1 that
// last read it has run.
int ring_acquire(rsp_plan* p, int* slot) {
    if (p->ring.empty()) {
        const int n = (p->nlanes + 1) * p->F;
        HIPCHK(hipStreamCreateWithFlags(&p->up_stream, hipStreamNonBlocking));
        p->ring.assign(n, nullptr);
        p->slot_ready.assign(n, nullptr);
        p->slot_free.assign(n, nullptr);
        p->slot_used.assign(n, 0);
        for (int i = 0; i < n; ++i) {
            int rc = p->dalloc_bytes(&p->ring[i], (size_t)p->g.C * p->g.cpitch * p->esz);
            if (rc) return rc;
            HIPCHK(hipEventCreateWithFlags(&p->slot_ready[i], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&p->slot_free[i], hipEventDisableTiming));
        }
    }
    const int s = p->ring_next;
    p->ring_next = (s + 1) % (int)p->ring.size();
    if (p->slot_used[s]) HIPCHK(hipStreamWaitEvent(p->up_stream, p->slot_free[s], 0));
    *slot = s;
    return RSP_OK;
}

int enqueue_frame(rsp_plan* p, const void* d_cube, int slot, int frame_idx, void* d_rdm = nullptr) {
    if (slot >= 0) {
        HIPCHK(hipEventRecord(p->slot_ready[slot], p->up_stream));
        p->slot_used[slot] = 1;
    }
    p->pend_in[p->npend] = d_cube;
    p->pend_rdm[p->npend] = d_rdm;
    p->pend_ids[p->npend] = frame_idx;
    p->pend_slot[p->npend] = slot;
    if (++p->npend == p->F) return flush_pending(p);
    return RSP_OK;
}

int ensure_stage(rsp_plan* p, size_t bytes) {
    if (p->h_stage_bytes >= bytes) return RSP_OK;
    if (p->h_stage) (void)hipHostFree(p->h_stage);
    p->h_stage = nullptr;
    HIPCHK(hipHostMalloc((void**)&p->h_stage, bytes, hipHostMallocDefault));
    p->h_stage_bytes = bytes;
    return RSP_OK;
}

// Copy a host cube (complex64 or complex128, nch channel slabs of N x P) into d_dst in the
// plan's precision (a converting copy only when the dtypes differ).
int upload_cube(rsp_plan* p, const void* cube, int dtype, int nch, void* d_dst, hipStream_t s) {
    if (dtype != RSP_C64 && dtype != RSP_C128) return fail(RSP_ERR_INVALID, "unknown dtype %d", dtype);
    const size_t slab = (size_t)p->g.N * p->g.P, elems = slab * nch;
    const bool f64 = p->g.prec == RSP_PREC_F64;
    const void* src = cube;
    if ((dtype == RSP_C128) != f64) {
        int rc = ensure_stage(p, elems * p->esz);
        if (rc) return rc;
        if (f64) {
            const float* a = (const float*)cube;
            double* o = (double*)p->h_stage;
            for (size_t i = 0; i < 2 * elems; ++i) o[i] = a[i];
        } else {
            const double* a = (const double*)cube;
            float* o = (float*)p->h_stage;
            for (size_t i = 0; i < 2 * elems; ++i) o[i] = (float)a[i];
        }
        src = p->h_stage;
    }
    HIPCHK(hipMemcpy2DAsync(d_dst, (size_t)p->g.cpitch * p->esz, src, slab * p->esz, slab * p->esz, nch,
                            hipMemcpyHostToDevice, s));   // channel slabs at cpitch
    HIPCHK(hipStreamSynchronize(s));   // the caller's buffer (or the staging buffer) is borrowed for the call
    return RSP_OK;
}

// [B][P][G] complex device maps -> MATLAB column-major [P x G x B] complex double
int rdm_to_matlab(rsp_plan* p, const void* d_map, double* out) {
    const int P = p->g.P, G = p->g.G, B = p->g.B;
    const size_t n = p->rdm_elems;
    std::vector<double> m(2 * n);
    if (p->g.prec == RSP_PREC_F64) {
        HIPCHK(hipMemcpy(m.data(), d_map, n * 16, hipMemcpyDeviceToHost));
    } else {
        std::vector<float> t(2 * n);
        HIPCHK(hipMemcpy(t.data(), d_map, n * 8, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < 2 * n; ++i) m[i] = t[i];
    }
    for (int b = 0; b < B; ++b)
        for (int v = 0; v < P; ++v)
            for (int r = 0; r < G; ++r) {
                const size_t i = ((size_t)b * P + v) * G + r;
                const size_t o = (size_t)v + (size_t)P * ((size_t)r + (size_t)G * b);
                out[2 * o] = m[2 * i];
                out[2 * o + 1] = m[2 * i + 1];
            }
    return RSP_OK;
}

// [B-1][P][G] real device maps (K3's S) -> MATLAB column-major [P x G x (B-1)] double
int smap_to_matlab(rsp_plan* p, const void* d_map, double* out) {
    const int P = p->g.P, G = p->g.G, NP = p->g.B - 1;
    const size_t n = (size_t)NP * P * G;
    std::vector<double> m(n);
    if (p->g.prec == RSP_PREC_F64) {
        HIPCHK(hipMemcpy(m.data(), d_map, n * 8, hipMemcpyDeviceToHost));
    } else {
        std::vector<float> t(n);
        HIPCHK(hipMemcpy(t.data(), d_map, n * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; ++i) m[i] = t[i];
    }
    for (int q = 0; q < NP; ++q)
        for (int v = 0; v < P; ++v)
            for (int r = 0; r < G; ++r)
                out[(size_t)v + (size_t)P * ((size_t)r + (size_t)G * q)] = m[((size_t)q * P + v) * G + r];
    return RSP_OK;
}

int run_sync_frame(rsp_plan* p, const void* d_in, int frame_idx, rsp_frame_out* out) {
    int rc = drain_all(p);
    if (rc) return rc;
    const size_t nres = p->results.size();
    Lane& L = p->lanes[0];
    const void* in[1] = {d_in};
    int ids[1] = {frame_idx};
    std::vector<std::vector<rsp_detection>> dets;
    void* smap = nullptr;
    if (out && out->cfar_maps && p->g.B > 1) {
        if (!p->d_smap && (rc = p->dalloc_bytes(&p->d_smap, (size_t)(p->g.B - 1) * p->g.P * p->g.G * p->rsz))) return rc;
        smap = p->d_smap;
    }
    void* rdm[1] = {L.rdm};
    if ((rc = launch_batch(p, L, in, ids, 1, smap, nullptr, out && out->rdm ? rdm : nullptr))) return rc;
    if ((rc = harvest(p, L, &dets))) return rc;
    FrameResult fr = p->results.back();
    p->results.resize(nres);   // synchronous frames do not enter the queue's result list
    p->last_dets = std::move(dets[0]);
    p->last_targets = fr.targets;
    if (out) {
        const std::vector<rsp_detection>& d = p->last_dets;
        out->n_dets = (int)d.size();
        if (out->dets) memcpy(out->dets, d.data(), sizeof(rsp_detection) * std::min<int>(out->dets_cap, (int)d.size()));
        out->n_targets = (int)fr.targets.size();
        if (out->targets)
            memcpy(out->targets, fr.targets.data(), sizeof(rsp_target) * std::min<int>(out->targets_cap, (int)fr.targets.size()));
        if (out->rdm && (rc = rdm_to_matlab(p, L.rdm, out->rdm))) return rc;
        if (smap && (rc = smap_to_matlab(p, smap, out->cfar_maps))) return rc;   // device-produced (fsf:184-187)
        if (out->dets && (int)d.size() > out->dets_cap)
            return fail(RSP_ERR_OVERFLOW, "%d detections exceed dets_cap %d (all of them: rsp_last_detections)",
                        (int)d.size(), out->dets_cap);
        if (out->targets && (int)fr.targets.size() > out->targets_cap)
            return fail(RSP_ERR_OVERFLOW, "%d targets exceed targets_cap %d (all of them: rsp_last_targets)",
                        (int)fr.targets.size(), out->targets_cap);
    }
    return RSP_OK;
}

const char* kStageNames[] = {"k1_dbf_mtd", "k2_pc", "k3_cfar"};

}  // namespace

// =========================================================================================
extern "C" {

const char* rsp_stage_name(int32_t s) { return (s >= 0 && s < 3) ? kStageNames[s] : "?"; }

int32_t rsp_plan_options_default(rsp_plan_options* o) {
    if (!o) return fail(RSP_ERR_INVALID, "null argument");
    o->device = 0;
    o->frames_per_launch = 1;
    o->precision = RSP_C128;
    o->flags = 0;
    return RSP_OK;
}

int32_t rsp_plan_create(const rsp_sig_config* cfg, const rsp_cfar_params* cfar, const rsp_cluster_params* cluster,
                        const rsp_precomputed* pre, int32_t device, int32_t frames_per_launch, rsp_plan** out) {
    rsp_plan_options o;
    rsp_plan_options_default(&o);
    o.device = device;
    o.frames_per_launch = frames_per_launch;
    return rsp_plan_create_ex(cfg, cfar, cluster, pre, &o, out);
}

int32_t rsp_plan_create_ex(const rsp_sig_config* cfg, const rsp_cfar_params* cfar, const rsp_cluster_params* cluster,
                           const rsp_precomputed* pre, const rsp_plan_options* opt, rsp_plan** out) {
    if (!cfg || !cfar || !cluster || !pre || !opt || !out) return fail(RSP_ERR_INVALID, "null argument");
    *out = nullptr;
    const int device = opt->device, frames_per_launch = opt->frames_per_launch;
    if (opt->precision != RSP_C64 && opt->precision != RSP_C128)
        return fail(RSP_ERR_INVALID, "precision must be RSP_C128 or RSP_C64, got %d", opt->precision);
    if (opt->flags & ~(RSP_PLAN_K1_TILED | RSP_PLAN_MONOPULSE_COMPLEX))
        return fail(RSP_ERR_INVALID, "unknown plan flags 0x%x", opt->flags);
    const int C = cfg->channel_num, B = cfg->beam_num, P = cfg->prtNum, N = cfg->point_PRT;
    const int g1 = pre->N_gate_narrow, g2 = pre->N_gate_medium, g3 = pre->N_gate_long, G = pre->N_total_gate;
    if (C < 1 || C > 32 || B < 1 || B > 16 || P < 2 || N < 2)
        return fail(RSP_ERR_INVALID, "bad sizes C=%d B=%d P=%d N=%d (1<=C<=32, 1<=B<=16)", C, B, P, N);
    if (P % 2) return fail(RSP_ERR_UNSUPPORTED, "odd prtNum %d (complex64 pulse pairs are loaded as 16 B)", P);
    if (g1 < 0 || g2 < 0 || g3 < 0 || G != g1 + g2 + g3 || G < 1) return fail(RSP_ERR_INVALID, "gate counts inconsistent");
    if (!pre->DBF_coeffs_data_C || !pre->MF_narrow || !pre->MF_medium_fft || !pre->MF_long_fft || !pre->MTD_win ||
        !pre->range_axis || !pre->velocity_axis || !pre->beam_angles_deg || (B > 1 && !pre->k_slopes_LUT))
        return fail(RSP_ERR_INVALID, "precomputed_data field missing");
    if (frames_per_launch < 1 || frames_per_launch > RSP_MAX_F)
        return fail(RSP_ERR_INVALID, "frames_per_launch must be 1..%d", RSP_MAX_F);
    const bool f64 = opt->precision == RSP_C128;
    const size_t esz = f64 ? 16 : 8;
    if ((size_t)C * N * P * esz >= ((size_t)1 << 31))
        return fail(RSP_ERR_UNSUPPORTED, "echo cube of %zu bytes: the kernels address one frame with 32-bit offsets (< 2 GB)",
                    (size_t)C * N * P * esz);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RSP_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(RSP_ERR_INVALID, "device %d out of range (%d devices)", device, ndev);
    HIPCHK(hipSetDevice(device));

    rsp_plan* p = new rsp_plan();
    p->device = device;
    p->F = frames_per_launch;
    p->cl = *cluster;
    p->c = cfg->c; p->fs = cfg->fs; p->wavelength = cfg->wavelength; p->d = cfg->element_spacing; p->prt = cfg->prt;
    p->p_signal_unscaled = pre->P_signal_unscaled;
    p->esz = esz;
    p->rsz = esz / 2;
    Geometry& g = p->g;
    g.prec = f64 ? RSP_PREC_F64 : RSP_PREC_F32;
    g.k1_tiled = (opt->flags & RSP_PLAN_K1_TILED) ? 1 : 0;
    g.mono_c = (opt->flags & RSP_PLAN_MONOPULSE_COMPLEX) ? 1 : 0;
    g.C = C; g.B = B; g.P = P; g.N = N; g.G = G;
    g.cpitch = N * P;
    g.refR = cfar->refCells_R; g.guardR = cfar->guardCells_R; g.refV = cfar->refCells_V; g.guardV = cfar->guardCells_V;
    g.T = cfar->T_CFAR;
    g.max_dets = 1;   // per launch: the lane's list capacity (launch_batch)
    {   // the most detections a frame can have: every cell under test of every beam pair (fsf:192-213)
        const int64_t nv = std::max(P - 2 * (g.refV + g.guardV), 0), nr = std::max(G - 2 * (g.refR + g.guardR), 0);
        p->det_bound = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)std::max(B - 1, 0) * nv * nr, 1 << 30));
    }
    if (hipDeviceGetAttribute(&g.ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) g.ncu = 0;
    auto bail = [&](int rc) { delete p; return rc; };
    if (g.refR < 1 || g.refV < 1 || g.guardR < 0 || g.guardV < 0) return bail(fail(RSP_ERR_INVALID, "bad CFAR window"));

    // ---- pulse-compression segments (fsf:105-126)
    std::vector<cd> H, twM;
    std::vector<int> tw_sizes, tw_offs;
    std::vector<double> taps;
    std::vector<Interval> need;
    if (g1 > 0) {
        SegDesc s{};
        s.type = 0;
        s.ga = 0; s.gb = g1;
        s.seg_lo = pre->seg_start_narrow - 1;
        if (s.seg_lo < 0 || s.seg_lo >= N) return bail(fail(RSP_ERR_INVALID, "seg_start_narrow out of range"));
        s.Ls = N - s.seg_lo;
        s.ntaps = pre->n_MF_narrow;
        s.delay = pre->fir_delay;
        if (s.ntaps < 1) return bail(fail(RSP_ERR_INVALID, "empty MF_narrow"));
        int lo = INT32_MAX, hi = -1;
        for (int gg = 0; gg < g1; ++gg) {
            int kk = (gg + s.delay) % s.Ls;
            if (kk < 0) kk += s.Ls;
            const int top = s.seg_lo + kk;
            const int bot = std::max(s.seg_lo, top - s.ntaps + 1);
            lo = std::min(lo, bot);
            hi = std::max(hi, top);
        }
        s.lo = lo; s.hi = hi;
        s.taps_off = (int)taps.size();
        for (int j = 0; j < s.ntaps; ++j) taps.push_back(pre->MF_narrow[j]);
        p->segs.push_back(s);
    }
    if (g2 > 0) {
        SegDesc s{};
        int rc = build_fft_segment(s, pre->MF_medium_fft, pre->N_fft_med, N, g1, g1 + g2, pre->seg_start_medium - 1, H,
                                   twM, tw_sizes, tw_offs, "medium");
        if (rc) return bail(rc);
        p->segs.push_back(s);
    }
    if (g3 > 0) {
        SegDesc s{};
        int rc = build_fft_segment(s, pre->MF_long_fft, pre->N_fft_long, N, g1 + g2, G, pre->seg_start_long - 1, H, twM,
                                   tw_sizes, tw_offs, "long");
        if (rc) return bail(rc);
        p->segs.push_back(s);
    }
    // K2 workgroup size in LDS points: a complex-double plan with a 2560-point block sizes every
    // workgroup for it (40 KB of LDS, no pads: 4 per CU, k2_pc's 128-VGPR budget), power-of-two
    // blocks then holding 2048 / M rows; otherwise RSP_K2_POINTS (4096: 2 per CU in complex double)
    g.k2_pts = RSP_K2_POINTS;
    for (auto& s : p->segs)
        if (f64 && s.type == 1 && s.M == 2560) g.k2_pts = RSP_K2_MIXPTS;
    for (auto& s : p->segs)   // a 4096-point block needs the 4096-point workgroups (2 per CU)
        if (s.type == 1 && s.M == 4096) g.k2_pts = RSP_K2_POINTS;
    // the narrow (direct-FIR) segment stages whole rows in the workgroup's LDS: when its window
    // does not fit a 2560-point workgroup the plan falls back to RSP_K2_POINTS workgroups (2 per
    // CU; k2_pc runs the 2560-point block in either sizing)
    for (auto& s : p->segs)
        if (s.type == 0 && g.k2_pts != RSP_K2_POINTS) {
            const int WP = s.hi - s.lo + 1 + s.ntaps - 1;
            if (WP + (s.ntaps + 1) / 2 > g.k2_pts) g.k2_pts = RSP_K2_POINTS;   // no pads at 2560
        }
    for (auto& s : p->segs) {
        if (s.seg_lo < 0 || s.seg_lo >= N) return bail(fail(RSP_ERR_INVALID, "segment start out of range"));
        if (s.hi >= s.lo) need.push_back({s.lo, s.hi});
        if (s.type == 1) {
            const int pts = (g.k2_pts == RSP_K2_POINTS) ? RSP_K2_POINTS : 2048;   // k2_pc's PTS
            s.rows_per_wg = s.M == 2560 ? 1 : std::max(1, pts / s.M);
        } else {
            // up to 8 rows per workgroup (measured best of 1/2/4/8 at x2), within the workgroup's
            // LDS: rows * WP complex + the taps (ntaps reals = ntaps / 2 complex)
            const int WP = s.hi - s.lo + 1 + s.ntaps - 1;   // staged row: ntaps - 1 leading zeros
            const int lds_c = g.k2_pts == RSP_K2_POINTS ? g.k2_pts + (g.k2_pts >> 5) : g.k2_pts;   // k2_pc's LDS
            s.rows_per_wg = std::max(1, std::min(8, (lds_c - (s.ntaps + 1) / 2) / WP));
            if (WP * s.rows_per_wg + (s.ntaps + 1) / 2 > lds_c)
                return bail(fail(RSP_ERR_UNSUPPORTED, "narrow segment window %d samples too long", s.hi - s.lo + 1));
        }
    }
    // union of needed fast-time windows -> compacted sample list (K1 processes only these)
    std::sort(need.begin(), need.end(), [](const Interval& a, const Interval& b) { return a.lo < b.lo; });
    std::vector<Interval> U;
    for (auto& iv : need) {
        if (!U.empty() && iv.lo <= U.back().hi + 1) U.back().hi = std::max(U.back().hi, iv.hi);
        else U.push_back(iv);
    }
    std::vector<int> nof;
    for (auto& iv : U) for (int n = iv.lo; n <= iv.hi; ++n) nof.push_back(n);
    g.nU = (int)nof.size();
    for (auto& s : p->segs) {
        if (s.hi < s.lo) { s.off = 0; continue; }
        s.off = (int)(std::lower_bound(nof.begin(), nof.end(), s.lo) - nof.begin());
    }
    // K1 tile: NT samples per [P][NT] slab.  complex64: LDS tile <= 80 KB (2 workgroups per
    // CU for the tiled K1; the persistent K1 double-buffers it) and B*NT*P <= 8192 (16 FFT
    // points per thread); complex128: the same bytes (NT halved) and B*NT*P <= 4096
    g.pow2P = is_pow2(P) && P >= 16 && P <= 512;   // Stockham range of k1_fft; else a DFT
    // other P = R Q (R = 2 or 4, Q odd >= 3; the reference's 332 = 4 x 83): the factored DFT
    // when one tile column per beam and its tables fit the LDS; otherwise the direct DFT
    g.rqR = g.rqQ = g.twq_elems = 0;
    if (!g.pow2P) {
        int R = 1;
        while (P % (2 * R) == 0) R *= 2;
        const int Q = P / R, Qh = (Q - 1) / 2;
        const int twq = (Qh + 1 + RQ_RK - 1) / RQ_RK * Qh * RQ_RK;
        if (R <= 4 && Q >= 3 && ((size_t)B * (P + 15) + twq + P) * esz <= 160 * 1024) {
            g.rqR = R;
            g.rqQ = Q;
            g.twq_elems = twq;
        }
    }
    // pow2: + one pad per 16 (K1_SH), see rsp_kernels.hip; factored DFT: the row stride in
    // P..P+15 whose pass-2 reads are conflict-free (rq_pick_stride)
    g.Ppad = g.pow2P ? P + P / 16 : (g.rqQ ? rq_pick_stride(g.rqR, g.rqQ, B) : P + 4);
    const int max_pts = f64 ? 4096 : 8192;
    const size_t tile_cap = f64 ? 72 * 1024 : 80 * 1024;
    const size_t tab_bytes = g.rqQ ? ((size_t)g.twq_elems + P) * esz : 0;   // k1_dft_rq's LDS tables
    g.NT = 8;
    while (g.NT > 1 && ((size_t)B * g.NT * g.Ppad * esz > tile_cap || (g.pow2P && B * g.NT * P > max_pts) ||
                        (size_t)B * g.NT * g.Ppad * esz + tab_bytes > 160 * 1024))
        g.NT >>= 1;
    if ((size_t)B * g.NT * g.Ppad * esz + tab_bytes > 160 * 1024 || (g.pow2P && B * g.NT * P > 8192))
        return bail(fail(RSP_ERR_UNSUPPORTED, "B*P too large for the slow-time FFT tile"));
    g.ntiles = (g.nU + g.NT - 1) / g.NT;
    // z chunks: NT samples (one K1 tile) per row slab
    g.NZ = g.NT;
    g.nzc = (g.nU + g.NZ - 1) / g.NZ;
    if ((int)U.size() > RSP_MAX_IVL) return bail(fail(RSP_ERR_UNSUPPORTED, "too many sample intervals"));
    g.nivl = (int)U.size();
    for (int q = 0, st = 0; q < g.nivl; ++q) {
        g.ivl_lo[q] = U[q].lo;
        g.ivl_start[q] = st;
        st += U[q].hi - U[q].lo + 1;
    }
    if (g.pow2P) g.logP = ilog2i(P);
    if (16 * (size_t)g.Ppad * esz > 160 * 1024 || (g.pow2P && 16 * P > 8192))
        return bail(fail(RSP_ERR_UNSUPPORTED, "prtNum %d too large", P));
    // K2 jobs
    const int rows_total = B * P;
    int wg = 0;
    for (size_t si = 0; si < p->segs.size(); ++si) {
        const SegDesc& s = p->segs[si];
        const int nwg = (rows_total + s.rows_per_wg - 1) / s.rows_per_wg;
        const int nbl = (s.type == 1) ? s.nblocks : 1;
        for (int blk = 0; blk < nbl; ++blk) {
            p->jobs.push_back(K2Job{(int)si, blk, wg, nwg});
            wg += nwg;
        }
    }
    g.nseg = (int)p->segs.size();
    g.njobs = (int)p->jobs.size();
    if (g.nseg > RSP_MAX_SEG || g.njobs > RSP_MAX_JOBS)
        return bail(fail(RSP_ERR_UNSUPPORTED, "%d overlap-save jobs exceed %d", g.njobs, RSP_MAX_JOBS));
    for (int q = 0; q < g.nseg; ++q) g.segs[q] = p->segs[q];
    for (int q = 0; q < g.njobs; ++q) g.jobs[q] = p->jobs[q];
    g.nwg_k2 = wg;
    // K3 tile: <= 64 KB of S per tile (>= 2 workgroups per CU); the fast path covers RT 32/64
    g.cfar_hR = (std::max(g.refR + g.guardR, 2) + 3) & ~3;   // halo, multiple of 4 (16-B tile loads)
    // tiles of RT range cells (64 complex single / 32 complex double: the fast path) x a band of
    // Doppler rows, <= RSP_K3_TILE_KB of S per tile (48 KB: 3 workgroups per CU; at P = 128 two
    // bands measured 78 vs 85 us per 8 x2 frames for one band at 2 workgroups per CU): at P = 128 one band holds every row; longer P (x4's 256)
    // splits the rows into bands, each with the rV + gV window rows on either side
    g.cfar_RT = p->rsz == 4 ? 64 : RSP_K3_RT_C128;
    // LDS row stride, 16-B aligned; complex double + 2 cells (bank spread, k3_cfar)
    // k3_cfar's compile-time path (the reference's 5/5/10/10) holds only the
    // band's own cells (its prefilter reads whichever range slice lies in the tile; the rare
    // survivors and S9 read the windows from the magnitude maps)
    const bool k3_nohalo = k3_fast_params(g);
    const int hx = k3_nohalo ? 0 : 2;
    g.cfar_W = ((g.cfar_RT + hx * g.cfar_hR + 3) & ~3) + (p->rsz == 8 ? 2 : 0);
    {
        const int hV = g.refV + g.guardV, ncut = std::max(P - 2 * hV, 1);
        const int hrows = k3_nohalo ? 0 : 2 * hV;
        const int rows_max = (int)((RSP_K3_TILE_KB * 1024) / ((size_t)g.cfar_W * p->rsz));
        if (rows_max - hrows < 1) return bail(fail(RSP_ERR_UNSUPPORTED, "CFAR window %d x %d exceeds the LDS tile", hV, g.cfar_hR));
        g.cfar_nband = (ncut + rows_max - hrows - 1) / (rows_max - hrows);
        g.cfar_VB = (ncut + g.cfar_nband - 1) / g.cfar_nband;
        g.cfar_rows = std::min(P, g.cfar_VB + hrows);
    }

    // ---- constants to the device, in the plan's precision
    int rc;
    const int bmax = B <= 4 ? 4 : (B <= 8 ? 8 : 16);
    const int cpad = C <= 8 ? 8 : (C <= 16 ? 16 : 32);   // CP of k1_dbf_mtd<T, BMAX, CP>
    // conj(W): y = x * W' (fsf:95), W column-major B x C
    auto wconj = [&](int b, int c) {
        const size_t i = (size_t)b + (size_t)B * c;
        return cd(pre->DBF_coeffs_data_C[2 * i], -pre->DBF_coeffs_data_C[2 * i + 1]);
    };
    // per-lane A operands of the DBF MFMA (k1_dbf_mtd): lane l holds A[row l&15][channel 4j + l>>4];
    // row m: beam mb*8 + (m&7), m<8 -> Re(y), m>=8 -> Im(y); y = sum_c conj(W[b][c]) x_c (fsf:95)
    const int mblk = bmax <= 8 ? 1 : 2, nj = cpad / 4;
    std::vector<double> atab((size_t)mblk * nj * 2 * 64, 0.0);
    for (int mb = 0; mb < mblk; ++mb)
        for (int j = 0; j < nj; ++j)
            for (int lane = 0; lane < 64; ++lane) {
                const int m = lane & 15, c = 4 * j + (lane >> 4), b = mb * 8 + (m & 7);
                double wr = 0, wi = 0;
                if (b < B && c < C) {
                    wr = wconj(b, c).real();
                    wi = wconj(b, c).imag();
                }
                const bool im = m >= 8;
                atab[((mb * nj + j) * 2 + 0) * 64 + lane] = im ? wi : wr;    // coefficient of Re(x_c)
                atab[((mb * nj + j) * 2 + 1) * 64 + lane] = im ? wr : -wi;   // coefficient of Im(x_c)
            }
    std::vector<cd> twPp, twP(P), twD;
    if (g.pow2P) build_pass_twiddles(g.logP, twPp);
    g.twPp_elems = (int)twPp.size();
    if (g.pow2P && P >= 64 && P <= 256)   // k1_fft_dif (k1_dif: P = 64 .. 256): compact pass-A twiddles, column-major [i][n2]
        for (int i = 0; i < 4; ++i)
            for (int n2 = 0; n2 < P / 16; ++n2) twD.push_back(root_of_unity((long long)n2 << i, P));
    for (int i = 0; i < P; ++i) twP[i] = root_of_unity(i, P);
    // k1_dft_rq's pass-2 table: [fset][n - 1][r] = (cos, sin)(2 pi k1 n / Q), k1 = RQ_RK fset + r
    // (zero past (Q - 1) / 2)
    std::vector<cd> twQ;
    if (g.rqQ) {
        const int Q = g.rqQ, Qh = (Q - 1) / 2, nfs = g.twq_elems / (Qh * RQ_RK);
        for (int fs = 0; fs < nfs; ++fs)
            for (int n = 1; n <= Qh; ++n)
                for (int r = 0; r < RQ_RK; ++r) {
                    const int k1 = fs * RQ_RK + r;
                    const cd w = k1 <= Qh ? root_of_unity((long long)k1 * n, Q) : cd(0.0, 0.0);
                    twQ.push_back(cd(w.real(), -w.imag()));   // exp(-i theta) -> (cos, sin) theta
                }
    }
    std::vector<double> win(pre->MTD_win, pre->MTD_win + P);
    std::vector<double> ra(pre->range_axis, pre->range_axis + G), va(pre->velocity_axis, pre->velocity_axis + P);
    std::vector<double> ang(pre->beam_angles_deg, pre->beam_angles_deg + B);
    std::vector<double> kl(std::max(B - 1, 1), 0.0);
    for (int i = 0; i + 1 < B; ++i) kl[i] = pre->k_slopes_LUT[i];
    DevConsts& k = p->k;
    double *dra, *dva, *dang, *dkl;
    if ((rc = p->upload_r(&k.Atab, atab)) || (rc = p->upload_c(&k.twP, twP)) || (rc = p->upload_c(&k.twPp, twPp)) || (rc = p->upload_c(&k.twD, twD)) || (rc = p->upload_c(&k.twQ, twQ)) ||
        (rc = p->upload_r(&k.win, win)) || (rc = p->upload_r(&k.taps, taps)) || (rc = p->upload_c(&k.H, H)) ||
        (rc = p->upload_c(&k.twM, twM)) || (rc = p->upload(&dra, ra)) || (rc = p->upload(&dva, va)) ||
        (rc = p->upload(&dang, ang)) || (rc = p->upload(&dkl, kl)))
        return bail(rc);
    k.range_axis = dra; k.velocity_axis = dva; k.beam_angles = dang; k.klut = dkl;
    {   // K2 dispatch order.  (1) Workgroups of a job covering adjacent rows form groups of gs
        // (below), at key (i + 1/2) / ngroups_j, so that the narrow FIR, medium and long jobs are
        // interleaved in proportion through the launch.  (2) Workgroups go to the 8 XCDs
        // round-robin by dispatch position, so the groups are laid out 8 at a time: positions
        // 8 (gs c + m) + x hold member m of group 8c + x -- every row of a group on one XCD, whose
        // L2 then serves the rest of every 128-B z line the first one fetched.  A z line holds
        // 128 / (NT esz) adjacent rows, a workgroup rows_per_wg of them, so gs = the most
        // workgroups one line spans over the jobs (x2: NT = 4, one-row long blocks -> 2; x4:
        // NT = 1 -> 8).  Workgroups left over go last.
        const int esz = 2 * p->rsz;
        int gs = 1;
        for (const K2Job& jb : p->jobs) {
            const int rw = std::max(p->segs[jb.seg].rows_per_wg, 1);
            gs = std::max(gs, std::min(8, 128 / std::max(rw * g.NZ * esz, 1)));
        }
        // (3) The overlap-save blocks of one row read overlapping sample windows (Lh - 1 samples
        // shared by neighbouring blocks: x4's long segment, 4 blocks): the groups of all blocks of
        // the same rows form one unit, placed on one XCD back to back, so that the shared lines
        // are L2 hits instead of second HBM fetches.  Units go to the XCD with the shortest queue
        // (round-robin when they are all the same size, x2) and the queues are interleaved:
        // dispatch position 8 s + x is the s-th workgroup of XCD x's queue.
        struct Unit { double key; std::vector<int> wgs; };
        std::vector<Unit> units;
        std::vector<int> single;
        for (int si = 0; si < (int)p->segs.size(); ++si) {
            std::vector<const K2Job*> blks;
            for (const K2Job& jb : p->jobs)
                if (jb.seg == si) blks.push_back(&jb);
            if (blks.empty()) continue;
            const int wc = blks[0]->wg_count, ng = wc / gs;   // every block of a segment covers all rows
            for (int i = 0; i < ng; ++i) {
                Unit u{(i + 0.5) / ng, {}};
                for (const K2Job* jb : blks)
                    for (int m = 0; m < gs; ++m) u.wgs.push_back(jb->wg_begin + gs * i + m);
                units.push_back(std::move(u));
            }
            for (const K2Job* jb : blks)
                for (int w = ng * gs; w < wc; ++w) single.push_back(jb->wg_begin + w);
        }
        std::stable_sort(units.begin(), units.end(), [](const Unit& x, const Unit& y) { return x.key < y.key; });
        std::vector<int> q[8];
        for (const Unit& u : units) {
            int x = 0;
            for (int c = 1; c < 8; ++c)
                if (q[c].size() < q[x].size()) x = c;
            q[x].insert(q[x].end(), u.wgs.begin(), u.wgs.end());
        }
        std::vector<int> order;
        size_t qmax = 0;
        for (auto& v : q) qmax = std::max(qmax, v.size());
        for (size_t sl = 0; sl < qmax; ++sl)
            for (int x = 0; x < 8; ++x)
                if (sl < q[x].size()) order.push_back(q[x][sl]);
        for (int w : single) order.push_back(w);
        if ((int)order.size() != g.nwg_k2) return bail(fail(RSP_ERR_INVALID, "K2 dispatch order covers %d of %d workgroups",
                                                            (int)order.size(), g.nwg_k2));
        int* dord;
        if ((rc = p->upload(&dord, order))) return bail(rc);
        k.k2order = dord;
    }
    k.deltaR = pre->deltaR; k.deltaV = pre->deltaV;
    if (pre->tx_pulse) {
        std::vector<double> tx(pre->tx_pulse, pre->tx_pulse + 2 * (size_t)N);
        if ((rc = p->upload(&p->d_tx, tx))) return bail(rc);
    }
    if ((rc = p->dalloc(&p->d_stab, (size_t)2 * RSP_MAX_SYNTH_TARGETS * (P + C)))) return bail(rc);
    p->z_elems = (size_t)B * g.nzc * g.NZ * P;
    p->rdm_elems = (size_t)B * P * G;
    g.Gp = (G + 3) & ~3;
    p->mag_elems = (size_t)B * P * g.Gp;
    if ((rc = p->dalloc_bytes(&p->d_cube, (size_t)std::max(C, B) * g.cpitch * esz))) return bail(rc);
    for (auto& L : p->lanes)
        if ((rc = setup_lane(p, L))) return bail(rc);
    *out = p;
    return RSP_OK;
}

int32_t rsp_set_stage_timing(rsp_plan* p, int32_t on) {
    if (!p) return fail(RSP_ERR_INVALID, "null plan");
    p->time_stages = on != 0;
    for (double& v : p->stage_ms) v = 0;
    p->stage_launches = p->stage_frames = 0;
    return RSP_OK;
}

int32_t rsp_stage_times(const rsp_plan* p, double* ms_sum, int32_t cap, int64_t* launches, int64_t* frames) {
    if (!p || !ms_sum || cap < 0) return fail(RSP_ERR_INVALID, "bad argument");
    for (int i = 0; i < std::min(cap, 3); ++i) ms_sum[i] = p->stage_ms[i];
    if (launches) *launches = p->stage_launches;
    if (frames) *frames = p->stage_frames;
    return RSP_OK;
}

int32_t rsp_plan_destroy(rsp_plan* plan) {
    delete plan;
    return RSP_OK;
}

int32_t rsp_query_sizes(const rsp_plan* p, rsp_sizes* s) {
    if (!p || !s) return fail(RSP_ERR_INVALID, "null argument");
    const Geometry& g = p->g;
    s->cube_elems = (int64_t)g.cpitch * g.C;
    s->rdm_elems = (int64_t)g.P * g.G * g.B;
    s->cfar_map_elems = (int64_t)g.P * g.G * std::max(g.B - 1, 0);
    s->P = g.P; s->N = g.N; s->C = g.C; s->B = g.B; s->G = g.G;
    s->used_samples = g.nU;
    s->max_detections = p->det_bound;
    s->n_stages = 3;
    s->precision = g.prec == RSP_PREC_F64 ? RSP_C128 : RSP_C64;
    s->elem_bytes = (int32_t)p->esz;
    return RSP_OK;
}

int32_t rsp_process_cube(rsp_plan* p, const void* cube, int32_t dtype, int32_t layout, int32_t frame_idx,
                         rsp_frame_out* out) {
    if (!p || !cube) return fail(RSP_ERR_INVALID, "null argument");
    if (layout != RSP_LAYOUT_PNC) return fail(RSP_ERR_UNSUPPORTED, "layout %d", layout);
    HIPCHK(hipSetDevice(p->device));
    int rc = drain_all(p);
    if (rc) return rc;
    if ((rc = upload_cube(p, cube, dtype, p->g.C, p->d_cube, p->lanes[0].stream))) return rc;
    return run_sync_frame(p, p->d_cube, frame_idx, out);
}

static int synth_into(rsp_plan* p, const rsp_target_in* t, int nt, int frame_idx, uint64_t seed, double p_noise,
                      void* d_cube, hipStream_t s, bool sync) {
    if (!p->d_tx) return fail(RSP_ERR_INVALID, "plan has no tx_pulse (synthesis path needs precomputed_data.tx_pulse)");
    if (nt < 0 || nt > RSP_MAX_SYNTH_TARGETS)
        return fail(RSP_ERR_INVALID, "0..%d targets supported, got %d", RSP_MAX_SYNTH_TARGETS, nt);
    SynthTargets tg{};
    for (int i = 0; i < nt; ++i) {   // fsf:51-72
        const double delay = 2.0 * t[i].Range / p->c;
        tg.t[i].delay = (int)mround(delay / (1.0 / p->fs));
        tg.t[i].fd_prt = 2.0 * t[i].Velocity / p->wavelength * p->prt;
        tg.t[i].amp = std::sqrt(std::pow(10.0, t[i].SNR_dB / 10.0) * p_noise / p->p_signal_unscaled);
        tg.t[i].dphi = 2.0 * M_PI * p->d * std::sin(t[i].ElevationAngle * M_PI / 180.0) / p->wavelength;
    }
    // the targets travel in the kernel arguments; the phasor tables are rewritten in stream order
    HIPCHK(launch_synth(p->g, p->d_tx, tg, nt, p->d_stab, frame_idx, seed, std::sqrt(p_noise / 2.0), d_cube, s));
    if (sync) HIPCHK(hipStreamSynchronize(s));   // the caller may read the cube from another stream
    return RSP_OK;
}

int32_t rsp_synthesize_device(rsp_plan* p, const rsp_target_in* t, int32_t nt, int32_t frame_idx, uint64_t seed,
                              double p_noise, void* d_cube) {
    if (!p || (!t && nt) || !d_cube) return fail(RSP_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(p->device));
    return synth_into(p, t, nt, frame_idx, seed, p_noise, d_cube, p->lanes[0].stream, true);
}

int32_t rsp_profile_synthesis(rsp_plan* p, const rsp_target_in* t, int32_t nt, int32_t iters, void* d_cube,
                              float* ms_out, int64_t* bytes_out) {
    if (!p || (!t && nt) || !d_cube || iters < 1 || !ms_out) return fail(RSP_ERR_INVALID, "bad argument");
    HIPCHK(hipSetDevice(p->device));
    int rc = drain_all(p);
    if (rc) return rc;
    hipStream_t s = p->lanes[0].stream;
    if ((rc = synth_into(p, t, nt, 1, 20250101, 1.0, d_cube, s, false))) return rc;   // warm-up
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, s));
    for (int i = 0; i < iters && !rc; ++i) rc = synth_into(p, t, nt, 1 + i, 20250101, 1.0, d_cube, s, false);
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    *ms_out = ms / iters;
    if (bytes_out) *bytes_out = (int64_t)p->g.C * p->g.N * p->g.P * (int64_t)p->esz;
    return RSP_OK;
}

int32_t rsp_process_targets(rsp_plan* p, const rsp_target_in* t, int32_t nt, int32_t frame_idx, uint64_t seed,
                            double p_noise, rsp_frame_out* out) {
    if (!p || (!t && nt)) return fail(RSP_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(p->device));
    int rc = drain_all(p);
    if (rc) return rc;
    // the frame runs on the same stream: no host synchronisation in between
    if ((rc = synth_into(p, t, nt, frame_idx, seed, p_noise, p->d_cube, p->lanes[0].stream, false))) return rc;
    return run_sync_frame(p, p->d_cube, frame_idx, out);
}

int32_t rsp_enqueue_device(rsp_plan* p, const void* d_cube, int32_t frame_idx) {
    if (!p || !d_cube) return fail(RSP_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(p->device));   // a host thread may drive plans on several devices
    return enqueue_frame(p, d_cube, -1, frame_idx);
}

int32_t rsp_enqueue_device_n(rsp_plan* p, const void* const* d_cubes, const int32_t* frame_idx, int32_t n) {
    if (!p || (n > 0 && (!d_cubes || !frame_idx)) || n < 0) return fail(RSP_ERR_INVALID, "bad argument");
    HIPCHK(hipSetDevice(p->device));
    for (int i = 0; i < n; ++i)   // all or nothing: no frame is queued when any pointer is bad
        if (!d_cubes[i]) return fail(RSP_ERR_INVALID, "cube %d is null", i);
    for (int i = 0; i < n; ++i) {
        int rc = enqueue_frame(p, d_cubes[i], -1, frame_idx[i]);
        if (rc) return rc;
    }
    return RSP_OK;
}

int32_t rsp_enqueue_device_rdm(rsp_plan* p, const void* d_cube, int32_t frame_idx, void* d_rdm) {
    if (!p || !d_cube || !d_rdm) return fail(RSP_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(p->device));
    return enqueue_frame(p, d_cube, -1, frame_idx, d_rdm);
}

int32_t rsp_enqueue_device_rdm_n(rsp_plan* p, const void* const* d_cubes, const int32_t* frame_idx, void* const* d_rdms,
                                 int32_t n) {
    if (!p || (n > 0 && (!d_cubes || !frame_idx || !d_rdms)) || n < 0) return fail(RSP_ERR_INVALID, "bad argument");
    HIPCHK(hipSetDevice(p->device));
    for (int i = 0; i < n; ++i)   // all or nothing: no frame is queued when any pointer is bad
        if (!d_cubes[i] || !d_rdms[i]) return fail(RSP_ERR_INVALID, "cube or map %d is null", i);
    for (int i = 0; i < n; ++i) {
        int rc = enqueue_frame(p, d_cubes[i], -1, frame_idx[i], d_rdms[i]);
        if (rc) return rc;
    }
    return RSP_OK;
}

int32_t rsp_enqueue_host(rsp_plan* p, const void* h_cube, int32_t dtype, int32_t frame_idx) {
    if (!p || !h_cube) return fail(RSP_ERR_INVALID, "null argument");
    if (dtype != (p->g.prec == RSP_PREC_F64 ? RSP_C128 : RSP_C64))
        return fail(RSP_ERR_INVALID, "rsp_enqueue_host: dtype %d differs from the plan precision (rsp_process_cube converts)",
                    dtype);
    HIPCHK(hipSetDevice(p->device));
    int s, rc;
    if ((rc = ring_acquire(p, &s))) return rc;
    // only the fast-time samples the chain reads (Geometry::ivl_*): per interval, the channel
    // slabs' [lo, lo + len) x P block, pitch N P
    const Geometry& g = p->g;
    const size_t row = (size_t)g.P * p->esz;
    for (int q = 0; q < g.nivl; ++q) {
        const int len = (q + 1 < g.nivl ? g.ivl_start[q + 1] : g.nU) - g.ivl_start[q];
        const size_t off = (size_t)g.ivl_lo[q] * row;
        HIPCHK(hipMemcpy2DAsync((char*)p->ring[s] + off, (size_t)g.cpitch * p->esz, (const char*)h_cube + off,
                                (size_t)g.N * row, (size_t)len * row, g.C, hipMemcpyHostToDevice, p->up_stream));
    }
    return enqueue_frame(p, p->ring[s], s, frame_idx);
}

int32_t rsp_host_alloc(rsp_plan* p, int64_t bytes, void** h_ptr) {
    if (!p || !h_ptr || bytes <= 0) return fail(RSP_ERR_INVALID, "bad argument");
    HIPCHK(hipSetDevice(p->device));
    *h_ptr = nullptr;
    if (hipHostMalloc(h_ptr, (size_t)bytes, hipHostMallocDefault) != hipSuccess)
        return fail(RSP_ERR_NOMEM, "hipHostMalloc(%lld bytes) failed", (long long)bytes);
    return RSP_OK;
}

int32_t rsp_host_free(rsp_plan* p, void* h_ptr) {
    if (!p) return fail(RSP_ERR_INVALID, "null argument");
    if (h_ptr) HIPCHK(hipHostFree(h_ptr));
    return RSP_OK;
}

int32_t rsp_process_targets_multi(rsp_plan* const* plans, int32_t n_plans, const rsp_target_in* const* targets,
                                  const int32_t* n_targets, const int32_t* frame_idx, int32_t n_frames, uint64_t seed,
                                  double p_noise, rsp_target* out, int32_t cap, int32_t* n_out) {
    if (!plans || n_plans < 1 || !targets || !n_targets || !frame_idx || n_frames < 0 || !out || cap < 0 || !n_out)
        return fail(RSP_ERR_INVALID, "bad argument");
    for (int i = 0; i < n_plans; ++i) {
        if (!plans[i]) return fail(RSP_ERR_INVALID, "plan %d is null", i);
        for (int j = 0; j < i; ++j)
            if (plans[j] == plans[i]) return fail(RSP_ERR_INVALID, "plan %d listed twice (one host thread per plan)", i);
        plans[i]->results_ready();
        if (!plans[i]->results.empty() || plans[i]->npend)
            return fail(RSP_ERR_INVALID, "plan %d has queued frames or uncleared results", i);
    }
    struct Work { int rc = RSP_OK; std::string err; };
    std::vector<Work> work(n_plans);
    auto run = [&](int i) {
        rsp_plan* p = plans[i];
        const int f0 = (int)((int64_t)n_frames * i / n_plans), f1 = (int)((int64_t)n_frames * (i + 1) / n_plans);
        auto body = [&]() -> int {
            HIPCHK(hipSetDevice(p->device));
            int rc;
            for (int j = f0; j < f1; ++j) {
                int s;
                if ((rc = ring_acquire(p, &s))) return rc;
                if ((rc = synth_into(p, targets[j], n_targets[j], frame_idx[j], seed, p_noise, p->ring[s], p->up_stream,
                                  false)))   // slot_ready orders K1 after it
                    return rc;
                if ((rc = enqueue_frame(p, p->ring[s], s, frame_idx[j]))) return rc;
            }
            if ((rc = drain_all(p))) return rc;
            for (int j = f0; j < f1; ++j) {   // results come back in enqueue order
                const FrameResult& r = p->results[j - f0];
                n_out[j] = (int32_t)r.targets.size();
                memcpy(out + (size_t)j * cap, r.targets.data(), sizeof(rsp_target) * std::min<size_t>(cap, r.targets.size()));
                if ((int)r.targets.size() > cap) return fail(RSP_ERR_OVERFLOW, "frame %d: %d targets > cap %d", frame_idx[j],
                                                             (int)r.targets.size(), cap);
            }
            p->results.clear();
            return RSP_OK;
        };
        work[i].rc = body();
        if (work[i].rc) {
            // leave the plan reusable: finish what was queued, then drop the partial share
            work[i].err = rsp_last_error();
            (void)drain_all(p);
            p->npend = 0;
            p->results.clear();
        }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < n_plans; ++i) th.emplace_back(run, i);
    run(0);
    for (auto& t : th) t.join();
    for (int i = 0; i < n_plans; ++i)
        if (work[i].rc) return fail(work[i].rc, "plan %d (device %d): %s", i, plans[i]->device, work[i].err.c_str());
    return RSP_OK;
}

int32_t rsp_drain(rsp_plan* p) {
    if (!p) return fail(RSP_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(p->device));
    return drain_all(p);
}

int32_t rsp_last_detections(const rsp_plan* p, rsp_detection* dets, int32_t cap, int32_t* n) {
    if (!p || !n || cap < 0 || (cap > 0 && !dets)) return fail(RSP_ERR_INVALID, "bad argument");
    const int m = (int)p->last_dets.size();
    *n = m;
    if (dets) memcpy(dets, p->last_dets.data(), sizeof(rsp_detection) * std::min(cap, m));
    if (dets && m > cap) return fail(RSP_ERR_OVERFLOW, "%d detections > cap %d", m, cap);
    return RSP_OK;
}

int32_t rsp_last_targets(const rsp_plan* p, rsp_target* targets, int32_t cap, int32_t* n) {
    if (!p || !n || cap < 0 || (cap > 0 && !targets)) return fail(RSP_ERR_INVALID, "bad argument");
    const int m = (int)p->last_targets.size();
    *n = m;
    if (targets) memcpy(targets, p->last_targets.data(), sizeof(rsp_target) * std::min(cap, m));
    if (targets && m > cap) return fail(RSP_ERR_OVERFLOW, "%d targets > cap %d", m, cap);
    return RSP_OK;
}

int32_t rsp_results_count(const rsp_plan* p, int32_t* n_frames, int64_t* n_targets) {
    if (!p) return fail(RSP_ERR_INVALID, "null argument");
    p->results_ready();
    int64_t nt = 0;
    for (auto& r : p->results) nt += (int64_t)r.targets.size();
    if (n_frames) *n_frames = (int32_t)p->results.size();
    if (n_targets) *n_targets = nt;
    return RSP_OK;
}

int32_t rsp_results_get(const rsp_plan* p, int32_t i, int32_t* frame_idx, rsp_target* targets, int32_t cap,
                        int32_t* n_targets, int32_t* n_dets) {
    if (!p) return fail(RSP_ERR_INVALID, "null argument");
    p->results_ready();
    if (i < 0 || i >= (int)p->results.size()) return fail(RSP_ERR_INVALID, "result index out of range");
    const FrameResult& r = p->results[i];
    if (frame_idx) *frame_idx = r.frame_idx;
    if (n_targets) *n_targets = (int32_t)r.targets.size();
    if (n_dets) *n_dets = r.n_dets;
    if (targets) memcpy(targets, r.targets.data(), sizeof(rsp_target) * std::min<size_t>(cap, r.targets.size()));
    if (targets && (int)r.targets.size() > cap) return fail(RSP_ERR_OVERFLOW, "cap too small");
    return RSP_OK;
}

int32_t rsp_results_rows(const rsp_plan* p, double* rows, int64_t cap, int64_t* n_rows) {
    if (!p || !n_rows) return fail(RSP_ERR_INVALID, "bad argument");
    p->results_ready();
    int64_t n = 0;
    for (const FrameResult& r : p->results) {
        const size_t nt = r.targets.size();
        for (size_t i = 0; i < std::max<size_t>(nt, 1); ++i, ++n) {
            if (!rows || n >= cap) continue;
            double* o = rows + 5 * n;
            o[0] = r.frame_idx;
            if (nt) {
                o[1] = r.targets[i].Range; o[2] = r.targets[i].Velocity; o[3] = r.targets[i].Angle; o[4] = r.targets[i].Power;
            } else {   // an empty frame stays visible as one NaN row
                o[1] = o[2] = o[3] = o[4] = std::nan("");
            }
        }
    }
    *n_rows = n;
    if (rows && n > cap) return fail(RSP_ERR_OVERFLOW, "%lld rows > cap %lld", (long long)n, (long long)cap);
    return RSP_OK;   // rows == NULL: a size query
}

int32_t rsp_results_clear(rsp_plan* p) {
    if (!p) return fail(RSP_ERR_INVALID, "null argument");
    p->results_ready();
    p->results.clear();
    return RSP_OK;
}

int32_t rsp_process_stage2(rsp_plan* p, const void* iq, int32_t dtype, double* mtd_out, double* pc_out) {
    if (!p || !iq) return fail(RSP_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(p->device));
    int rc = drain_all(p);
    if (rc) return rc;
    Lane& L = p->lanes[0];
    Geometry gs = p->g;
    gs.C = gs.B;   // input channels are the beams; K1 transposes only (no DBF, no MTD)
    if ((rc = upload_cube(p, iq, dtype, gs.B, p->d_cube, L.stream))) return rc;
    if (!p->d_aux && (rc = p->dalloc_bytes(&p->d_aux, p->rdm_elems * p->esz))) return rc;
    const void* in[1] = {p->d_cube};
    void* rdm[1] = {L.rdm};
    const FramePtrs fp = lane_ptrs(p, L, in, 1, rdm);
    HIPCHK(launch_k1(gs, p->k, fp, 1, 0, L.stream));
    HIPCHK(launch_k2(gs, p->k, fp, 1, gs.B * gs.P, L.stream));      // PC rows (b, m) -> L.rdm
    HIPCHK(launch_mtd_cols(gs, p->k, L.rdm, p->d_aux, L.stream));  // S7 over pulses
    HIPCHK(hipStreamSynchronize(L.stream));
    if (pc_out && (rc = rdm_to_matlab(p, L.rdm, pc_out))) return rc;
    if (mtd_out && (rc = rdm_to_matlab(p, p->d_aux, mtd_out))) return rc;
    return RSP_OK;
}

int32_t rsp_process_stage2_gated(rsp_plan* p, const void* iq, int32_t dtype, int32_t n_gated, const int32_t* cols,
                                 double* mtd_out, double* pc_out) {
    if (!p || !iq) return fail(RSP_ERR_INVALID, "null argument");
    if (dtype != RSP_C64 && dtype != RSP_C128) return fail(RSP_ERR_INVALID, "unknown dtype %d", dtype);
    static const int32_t kRefCols[6] = {83, 310, 311, 1033, 1034, 3486};   // main_simulate_echoes_with_array_v2.m:257-264
    const int32_t* c = cols ? cols : kRefCols;
    const int P = p->g.P, N = p->g.N, B = p->g.B;
    int total = 0;
    for (int k = 0; k < 3; ++k) {
        if (c[2 * k] < 1 || c[2 * k + 1] < c[2 * k] || c[2 * k + 1] > N)
            return fail(RSP_ERR_INVALID, "gate columns %d..%d of segment %d outside the %d-sample PRT", c[2 * k],
                        c[2 * k + 1], k, N);
        if (k > 0 && c[2 * k] <= c[2 * k - 1])   // ascending and disjoint, like v2:257-264
            return fail(RSP_ERR_INVALID, "gate columns of segment %d (%d..%d) overlap or precede segment %d (..%d)", k,
                        c[2 * k], c[2 * k + 1], k - 1, c[2 * k - 1]);
        total += c[2 * k + 1] - c[2 * k] + 1;
    }
    if (total != n_gated) return fail(RSP_ERR_INVALID, "gated input has %d columns, the gate columns cover %d", n_gated, total);
    // put the gated columns back at their PRT positions (zeros elsewhere): [P x N x B]
    const size_t es = dtype == RSP_C128 ? 16 : 8, colb = (size_t)P * es;
    std::vector<unsigned char> full((size_t)N * B * colb, 0);
    const unsigned char* src = static_cast<const unsigned char*>(iq);
    for (int b = 0; b < B; ++b) {
        int ng = 0;
        for (int k = 0; k < 3; ++k)
            for (int col = c[2 * k] - 1; col < c[2 * k + 1]; ++col, ++ng)
                memcpy(&full[((size_t)b * N + col) * colb], src + ((size_t)b * n_gated + ng) * colb, colb);
    }
    return rsp_process_stage2(p, full.data(), dtype, mtd_out, pc_out);
}

int32_t rsp_profile_stages(rsp_plan* p, const void* const* d_cubes, int32_t n_cubes, int32_t iters, float* ms_out,
                           int64_t* bytes_out, int32_t cap, int32_t* frames_out) {
    return rsp_profile_stages_rdm(p, d_cubes, n_cubes, nullptr, iters, ms_out, bytes_out, cap, frames_out);
}

int32_t rsp_profile_stages_rdm(rsp_plan* p, const void* const* d_cubes, int32_t n_cubes, void* const* d_rdms,
                               int32_t iters, float* ms_out, int64_t* bytes_out, int32_t cap, int32_t* frames_out) {
    if (!p || !d_cubes || n_cubes < 1 || iters < 1) return fail(RSP_ERR_INVALID, "bad argument");
    HIPCHK(hipSetDevice(p->device));
    int rc = drain_all(p);
    if (rc) return rc;
    Lane& L = p->lanes[0];
    const int nf = std::min(n_cubes, p->F);
    for (int f = 0; f < nf && d_rdms; ++f)   // d_rdms holds (at least) one map per frame of the batch
        if (!d_rdms[f]) return fail(RSP_ERR_INVALID, "map %d is null (d_rdms needs min(n_cubes, F) maps)", f);
    // batches rotate over all n_cubes cubes (cube (j nf + f) mod n_cubes in batch j), so that a
    // ring larger than the 256 MiB Infinity Cache makes K1 read its input from HBM as in the queue
    const int nsets = (n_cubes + nf - 1) / nf;
    std::vector<FramePtrs> fps(nsets);
    for (int j = 0; j < nsets; ++j) {
        const void* in[RSP_MAX_F];
        for (int f = 0; f < nf; ++f) in[f] = d_cubes[(j * nf + f) % n_cubes];
        fps[j] = lane_ptrs(p, L, in, nf, d_rdms);   // as the queue: complex RDM stores only into d_rdms
    }
    const Geometry& g = p->g;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    for (int s = 0; s < 3 && s < cap; ++s) {
        int it = 0;
        auto run = [&]() -> hipError_t {
            const FramePtrs& fj = fps[it++ % nsets];
            if (s == 0) return launch_k1(g, p->k, fj, nf, 3, L.stream);
            if (s == 1) return launch_k2(g, p->k, fj, nf, g.B * g.P, L.stream);
            // counts are zeroed by K1 in the pipeline; here by a tiny 2-D memset per launch
            hipError_t e = hipMemset2DAsync(L.dets, sizeof(DevDet) * (L.dcap + 1), 0, sizeof(int), nf, L.stream);
            Geometry g3 = g;
            g3.max_dets = L.dcap;
            return e != hipSuccess ? e : launch_k3(g3, p->k, fj, nf, L.stream);
        };
        HIPCHK(run());
        HIPCHK(hipEventRecord(e0, L.stream));
        for (int i = 0; i < iters; ++i) HIPCHK(run());
        HIPCHK(hipEventRecord(e1, L.stream));
        HIPCHK(hipEventSynchronize(e1));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        if (ms_out) ms_out[s] = ms / iters;
    }
    if (frames_out) *frames_out = nf;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (bytes_out) {   // algorithmic bytes per launch (nf frames); DESIGN.md "Measurement"
        const int64_t es = (int64_t)p->esz, rs = (int64_t)p->rsz;   // complex / real element bytes
        const int64_t cube = (int64_t)g.C * g.nU * g.P * es;       // used fast-time samples
        const int64_t z = (int64_t)g.B * g.nU * g.P * es;          // Doppler-domain rows
        const int64_t mag = (int64_t)g.B * g.P * g.G * rs;         // |RD| map (the RDM stays on chip)
        if (cap > 0) bytes_out[0] = nf * (cube + z);
        // the complex RD map, when written: into d_rdms, or (complex-ratio monopulse) into the
        // lane's own map, which K3 then reads only at the detected cells (2 values per detection,
        // not a map-sized stream, so K3's bytes stay the magnitude maps)
        const int64_t rdm = (d_rdms || g.mono_c) ? (int64_t)g.B * g.P * g.G * es : 0;
        if (cap > 1) bytes_out[1] = nf * (z + mag + rdm);
        if (cap > 2) bytes_out[2] = nf * k3_map_bytes(g, (int)rs);   // the rows under test (rsp_internal.h)
    }
    return RSP_OK;
}

int32_t rsp_hbm_copy_probe(int32_t device, int64_t bytes, int32_t iters, double* gbps) {
    if (!gbps || bytes < (1 << 20) || iters < 1) return fail(RSP_ERR_INVALID, "bad argument");
    HIPCHK(hipSetDevice(device));
    int ncu = 0;
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
    const size_t n16 = (size_t)bytes / 16;
    void *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, n16 * 16) != hipSuccess) return fail(RSP_ERR_NOMEM, "hipMalloc(%lld) failed", (long long)bytes);
    if (hipMalloc(&b, n16 * 16) != hipSuccess) {
        (void)hipFree(a);
        return fail(RSP_ERR_NOMEM, "hipMalloc(%lld) failed", (long long)bytes);
    }
    hipEvent_t e0, e1;
    hipError_t e = hipMemset(a, 0, n16 * 16);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    float ms = 0.f;
    if (e == hipSuccess) {
        for (int i = 0; i < 3 && e == hipSuccess; ++i) e = launch_stream_copy(a, b, n16, ncu, nullptr);
        if (e == hipSuccess) e = hipEventRecord(e0, nullptr);
        for (int i = 0; i < iters && e == hipSuccess; ++i) e = launch_stream_copy(a, b, n16, ncu, nullptr);
        if (e == hipSuccess) e = hipEventRecord(e1, nullptr);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    (void)hipFree(a);
    (void)hipFree(b);
    if (e != hipSuccess) return fail(RSP_ERR_DEVICE, "copy probe: %s", hipGetErrorString(e));
    *gbps = 2.0 * (double)(n16 * 16) / (ms * 1e-3 / iters) / 1e9;
    return RSP_OK;
}

int32_t rsp_device_alloc(rsp_plan* p, int64_t bytes, void** d) {
    if (!p || !d || bytes <= 0) return fail(RSP_ERR_INVALID, "bad argument");
    HIPCHK(hipSetDevice(p->device));
    if (hipMalloc(d, bytes) != hipSuccess) return fail(RSP_ERR_NOMEM, "hipMalloc(%lld) failed", (long long)bytes);
    return RSP_OK;
}
int32_t rsp_device_free(rsp_plan* p, void* d) {
    if (!p) return fail(RSP_ERR_INVALID, "null plan");
    HIPCHK(hipFree(d));
    return RSP_OK;
}
int32_t rsp_device_upload(rsp_plan* p, void* d, const void* h, int64_t bytes) {
    if (!p || !d || !h) return fail(RSP_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(p->device));
    HIPCHK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    return RSP_OK;
}
int32_t rsp_device_download(rsp_plan* p, void* h, const void* d, int64_t bytes) {
    if (!p || !d || !h) return fail(RSP_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(p->device));
    HIPCHK(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
    return RSP_OK;
}
int32_t rsp_device_sync(rsp_plan* p) {
    if (!p) return fail(RSP_ERR_INVALID, "null plan");
    HIPCHK(hipSetDevice(p->device));
    HIPCHK(hipDeviceSynchronize());
    return RSP_OK;
}

}  // extern "C"
