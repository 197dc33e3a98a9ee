// Host-only driver of librsp's plain-C++ parts (rsp_mat.cpp, rsp_host.cpp) for the
// AddressSanitizer / UBSan build of tests/test_host_asan.py.  Status codes are ignored: only
// memory errors (reported by the sanitizers, exit code != 0) fail the test.
//   host_fuzz mat FILE...     every MAT entry point on every file
//   host_fuzz cluster SEED    S10/S11 and inter-frame clustering on random lists
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rsp.h"

static int mat(int argc, char** argv) {
    for (int i = 2; i < argc; ++i) {
        rsp_mat_var vars[8];
        int32_t nv = 0;
        rsp_mat_list(argv[i], vars, 8, &nv);
        for (int v = 0; v < nv && v < 8; ++v) {
            std::vector<double> d(64);
            std::vector<float> f(64);
            std::vector<char> c(64);
            rsp_mat_read(argv[i], vars[v].name, RSP_MAT_OUT_F64, d.data(), (int64_t)d.size());
            rsp_mat_read(argv[i], vars[v].name, RSP_MAT_OUT_F32, f.data(), (int64_t)f.size());
            rsp_mat_read(argv[i], vars[v].name, RSP_MAT_OUT_CHAR, c.data(), (int64_t)c.size());
        }
        int32_t dims[3] = {0, 0, 0}, na = 0;
        double ang[16];
        std::vector<double> cube(2 * 4096);
        rsp_mat_load_frame(argv[i], RSP_C128, cube.data(), 4096, dims, ang, 16, &na);
        rsp_mat_load_frame(argv[i], RSP_C64, cube.data(), 4096, dims, ang, 16, &na);
        rsp_mat_load_frame(argv[i], RSP_C128, nullptr, 0, dims, nullptr, 0, &na);
    }
    return 0;
}

static int cluster(unsigned seed) {
    std::mt19937_64 g(seed);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    rsp_cluster_params cp = {30.0, 0.4, 5.0};
    for (int rep = 0; rep < 20; ++rep) {
        const int n = (int)(u(g) * 3000);
        std::vector<rsp_detection> d(n);
        for (int i = 0; i < n; ++i) {
            const int c = (int)(u(g) * 8);
            d[i] = rsp_detection{(int32_t)(16 + u(g) * 90), (int32_t)(16 + u(g) * 2000), (int32_t)(1 + u(g) * 7), 0,
                                 1 + 99 * u(g), 1000.0 * c + 50 * u(g), 5.0 + 0.5 * c + 0.3 * u(g), 3.0 * c + 3 * u(g)};
        }
        std::vector<rsp_target> out(64);
        int32_t no = 0;
        rsp_cluster_detections(d.data(), n, &cp, out.data(), (int32_t)out.size(), &no);   // may overflow cap: status only
        std::vector<rsp_track_point> pts(n);
        for (int i = 0; i < n; ++i)
            pts[i] = rsp_track_point{d[i].Range, d[i].Velocity, d[i].Angle, d[i].amp, 10 * u(g), (int32_t)(u(g) * 20), 0};
        rsp_inter_frame_params ip = {30.0, 1.0, 2.0, 3.0, 2, 0};
        std::vector<rsp_track> tr(32);
        rsp_inter_frame_cluster(pts.data(), n, &ip, tr.data(), (int32_t)tr.size(), &no);
    }
    rsp_cluster_detections(nullptr, 0, &cp, nullptr, 0, nullptr);
    int32_t no = 0;
    rsp_cluster_detections(nullptr, 0, &cp, nullptr, 0, &no);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && !strcmp(argv[1], "mat")) return mat(argc, argv);
    if (argc >= 3 && !strcmp(argv[1], "cluster")) return cluster((unsigned)atoi(argv[2]));
    fprintf(stderr, "usage: host_fuzz mat FILE... | cluster SEED\n");
    return 2;
}
