// Instruction census of one K2 job type (compiled with -S only, never linked): the product's
// rsp_kernels.hip plus two kernels that run a single overlap-save block type on the queue's
// path (no complex RD map), so that tools/ab/census.sh can count its instructions and registers.
#include "../../radar-signal-simulation-and-target-detection_amd/csrc/rsp_kernels.hip"

namespace {
template <int KIND>   // 1: the 2560-point mixed-radix block, 2: a 1024-point block
__global__ __launch_bounds__(K2_THREADS, RSP_K2_MINB) void k2_census(Geometry g, DevConsts k, FramePtrs fp,
                                                                     int rows_total) {
    typedef cx<double> V;
    V* L = reinterpret_cast<V*>(rsp_lds);
    const K2Job job = g.jobs[blockIdx.z];
    const SegDesc& sd = g.segs[job.seg];
    const int row0 = ((int)blockIdx.x - job.wg_begin) * sd.rows_per_wg;
    const V* z = static_cast<const V*>(fp.z[blockIdx.y]);
    double* mag = static_cast<double*>(fp.mag[blockIdx.y]);
    if constexpr (KIND == 1) k2_fft_job_mix<double, 2560, 10>(g, k, sd, job, z, nullptr, mag, row0, rows_total, L);
    else k2_fft_job<double, 10>(g, k, sd, job, z, nullptr, mag, row0, rows_total, L);
}
template __global__ void k2_census<1>(Geometry, DevConsts, FramePtrs, int);
template __global__ void k2_census<2>(Geometry, DevConsts, FramePtrs, int);
}  // namespace
