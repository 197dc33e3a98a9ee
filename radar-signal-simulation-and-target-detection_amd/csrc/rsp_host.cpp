// rsp_host.cpp -- host-only parts of librsp (plain C++, no HIP): the error sink of the C-ABI,
// the S10/S11 two-stage clustering of fun_process_single_frame.m:302-407 and the inter-frame
// track association of main_simulate_echoes_with_array_v8_3.m:253-352.  Built with the host
// compiler, so the CPU test suite can also build it under AddressSanitizer
// (tests/test_host_asan.py).
#include "rsp.h"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int vfail(int code, const char* fmt, va_list ap) {
    char buf[1024];
    vsnprintf(buf, sizeof buf, fmt, ap);
    g_err = buf;
    return code;
}

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

}  // namespace

// Error sink shared with the other translation units (not exported).
__attribute__((visibility("hidden"))) int rsp_set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

namespace {

// ---- S10 / S11 on the host (fsf:302-407) ---------------------------------------------
// The reference labels clusters with a BFS that scans every point for every visited point
// (O(n^2)).  Its clusters are exactly the connected components of the "close" relation, and
// cluster k is the component whose smallest index is the k-th smallest such index.  We find
// the same components with union-find over the edges of a sweep in Range order (close()
// requires |dR| <= max_range_sep, so no other pair can be an edge) and number them the same
// way; member sums then run in index order like the reference's cluster_mask loops.
struct DSU {
    std::vector<int> p;
    explicit DSU(int n) : p(n) { for (int i = 0; i < n; ++i) p[i] = i; }
    int find(int x) {
        while (p[x] != x) x = p[x] = p[p[x]];
        return x;
    }
    void unite(int a, int b) {
        a = find(a); b = find(b);
        if (a != b) p[a < b ? b : a] = a < b ? a : b;
    }
};

template <class Item, class Close>
int component_labels(const std::vector<Item>& it, double rsep, Close close, std::vector<int>& ids) {
    const int n = (int)it.size();
    std::vector<int> ord(n);
    for (int i = 0; i < n; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return it[a].Range < it[b].Range; });
    DSU d(n);
    for (int x = 0; x < n; ++x)
        for (int y = x + 1; y < n && it[ord[y]].Range - it[ord[x]].Range <= rsep; ++y)
            if (close(it[ord[x]], it[ord[y]])) d.unite(ord[x], ord[y]);
    ids.assign(n, 0);
    std::vector<int> lab(n, 0);
    int cur = 0;
    for (int i = 0; i < n; ++i) {
        const int r = d.find(i);
        if (!lab[r]) lab[r] = ++cur;
        ids[i] = lab[r];
    }
    return cur;
}

void cluster_frame_impl(const rsp_cluster_params& cp, std::vector<rsp_detection>& dets,
                   std::vector<rsp_target>& final_targets) {
    // reference order of all_raw_detections: pair, then find() column-major (r, v)  (fsf:181,215-221)
    std::sort(dets.begin(), dets.end(), [](const rsp_detection& a, const rsp_detection& b) {
        if (a.pair_idx != b.pair_idx) return a.pair_idx < b.pair_idx;
        if (a.r_idx != b.r_idx) return a.r_idx < b.r_idx;
        return a.v_idx < b.v_idx;
    });
    final_targets.clear();
    const int n = (int)dets.size();
    if (!n) return;
    std::vector<int> ids;
    const int n1 = component_labels(dets, cp.max_range_sep, [&](const rsp_detection& a, const rsp_detection& b) {
        return std::fabs(a.Range - b.Range) <= cp.max_range_sep && std::fabs(a.Velocity - b.Velocity) <= cp.max_vel_sep &&
               std::fabs(a.Angle - b.Angle) <= cp.max_angle_sep;
    }, ids);
    std::vector<rsp_target> st1(n1, rsp_target{0, 0, 0, 0});
    std::vector<double> sr(n1, 0.0), sv(n1, 0.0), sa(n1, 0.0);
    for (int i = 0; i < n; ++i) st1[ids[i] - 1].Power += dets[i].amp;   // power-weighted means (fsf:341-351)
    for (int i = 0; i < n; ++i) {
        const int c = ids[i] - 1;
        sr[c] += dets[i].Range * dets[i].amp;
        sv[c] += dets[i].Velocity * dets[i].amp;
        sa[c] += dets[i].Angle * dets[i].amp;
    }
    for (int c = 0; c < n1; ++c) {
        const double tp = st1[c].Power;
        st1[c] = rsp_target{sr[c] / tp, sv[c] / tp, sa[c] / tp, tp};
    }
    const int n2 = component_labels(st1, cp.max_range_sep, [&](const rsp_target& a, const rsp_target& b) {
        return std::fabs(a.Range - b.Range) <= cp.max_range_sep && std::fabs(a.Velocity - b.Velocity) <= cp.max_vel_sep;
    }, ids);
    std::vector<int> win(n2, -1);   // winner-take-all, first max in index order (fsf:393-406)
    for (int i = 0; i < n1; ++i) {
        int& w = win[ids[i] - 1];
        if (w < 0 || st1[i].Power > st1[w].Power) w = i;
    }
    for (int c = 0; c < n2; ++c) final_targets.push_back(st1[win[c]]);
}

}  // namespace

__attribute__((visibility("hidden"))) void rsp_cluster_frame(const rsp_cluster_params& cp, std::vector<rsp_detection>& dets,
                                                             std::vector<rsp_target>& final_targets) {
    cluster_frame_impl(cp, dets, final_targets);
}

extern "C" {

int32_t rsp_abi_version(void) { return RSP_ABI_VERSION; }
const char* rsp_last_error(void) { return g_err.c_str(); }

int32_t rsp_cluster_detections(const rsp_detection* dets, int32_t n, const rsp_cluster_params* cp,
                               rsp_target* out, int32_t cap, int32_t* n_out) {
    if ((!dets && n) || n < 0 || !cp || !n_out) return fail(RSP_ERR_INVALID, "bad argument");
    std::vector<rsp_detection> d(dets, dets + n);
    std::vector<rsp_target> t;
    cluster_frame_impl(*cp, d, t);
    *n_out = (int32_t)t.size();
    if (out) memcpy(out, t.data(), sizeof(rsp_target) * std::min<size_t>(cap, t.size()));
    if ((int)t.size() > cap) return fail(RSP_ERR_OVERFLOW, "%d targets exceed cap %d", (int)t.size(), cap);
    return RSP_OK;
}

// Inter-frame track association (main_simulate_echoes_with_array_v8_3.m:253-352): the BFS
// of :270-304 over the 5-D gate (|dR|, |dV|, |dAz|, |dEl|, |dFrame|) = connected components
// numbered by smallest member index (component_labels, sweep in Range order); then per cluster,
// members in log order (:312-335): total power, first-max winner (R, V, El, Power), power-weighted
// azimuth, first/last frame, count.
int32_t rsp_inter_frame_cluster(const rsp_track_point* log, int32_t n, const rsp_inter_frame_params* gp,
                                rsp_track* out, int32_t cap, int32_t* n_out) {
    if ((!log && n) || n < 0 || !gp || !n_out || cap < 0) return fail(RSP_ERR_INVALID, "bad argument");
    std::vector<rsp_track_point> pts(log, log + n);
    std::vector<int> ids;
    const rsp_inter_frame_params g = *gp;
    const int nc = n ? component_labels(pts, g.Gate_R, [&](const rsp_track_point& a, const rsp_track_point& b) {
        return std::fabs(a.Range - b.Range) <= g.Gate_R && std::fabs(a.Velocity - b.Velocity) <= g.Gate_V &&
               std::fabs(a.iAntAngle - b.iAntAngle) <= g.Gate_Az && std::fabs(a.Angle - b.Angle) <= g.Gate_El &&
               std::abs(a.iFrame - b.iFrame) <= g.Max_Frame_Gap;
    }, ids) : 0;
    std::vector<rsp_track> tr(nc);
    std::vector<double> ptot(nc, 0.0), paz(nc, 0.0);
    std::vector<int> win(nc, -1);
    for (int i = 0; i < n; ++i) {   // members in log order, like detection_log(cluster_mask)
        const int c = ids[i] - 1;
        rsp_track& t = tr[c];
        ptot[c] += pts[i].Power;
        paz[c] += pts[i].iAntAngle * pts[i].Power;
        if (win[c] < 0) {
            t.FirstFrame = t.LastFrame = pts[i].iFrame;
            t.NumPoints = 0;
        }
        if (win[c] < 0 || pts[i].Power > pts[win[c]].Power) win[c] = i;   // [max_power, idx_winner] = max(powers)
        t.FirstFrame = std::min(t.FirstFrame, pts[i].iFrame);
        t.LastFrame = std::max(t.LastFrame, pts[i].iFrame);
        ++t.NumPoints;
    }
    for (int c = 0; c < nc; ++c) {
        const rsp_track_point& w = pts[win[c]];
        tr[c].Range = w.Range;
        tr[c].Velocity = w.Velocity;
        tr[c].Angle = w.Angle;
        tr[c].Azimuth = paz[c] / ptot[c];
        tr[c].Power = w.Power;
        tr[c].reserved = 0;
    }
    *n_out = nc;
    if (out) memcpy(out, tr.data(), sizeof(rsp_track) * std::min<size_t>(cap, tr.size()));
    if (nc > cap) return fail(RSP_ERR_OVERFLOW, "%d tracks exceed cap %d", nc, cap);
    return RSP_OK;
}

}  // extern "C"
