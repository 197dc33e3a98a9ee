/* rsp_cplx_pack.h -- complex data between MATLAB's split storage (separate real and imaginary
 * blocks: the pre-R2018a C Matrix API, mxGetPr / mxGetPi) and the interleaved (re, im) pairs
 * include/rsp.h takes and returns (SURVEY 8(b) "Layout").  Plain C, no MATLAB types: the CPU
 * test suite compiles and runs these directly (tests/native/test_cplx_pack.c). */
#ifndef RSP_CPLX_PACK_H
#define RSP_CPLX_PACK_H
#include <stddef.h>

/* out[2i] = re[i], out[2i+1] = im[i] (im == NULL: a real array, imaginary parts 0) */
static inline void rsp_interleave_f64(const double* re, const double* im, size_t n, double* out) {
    size_t i;
    for (i = 0; i < n; ++i) {
        out[2 * i] = re[i];
        out[2 * i + 1] = im ? im[i] : 0.0;
    }
}
static inline void rsp_interleave_f32(const float* re, const float* im, size_t n, float* out) {
    size_t i;
    for (i = 0; i < n; ++i) {
        out[2 * i] = re[i];
        out[2 * i + 1] = im ? im[i] : 0.0f;
    }
}
/* re[i] = in[2i], im[i] = in[2i+1] */
static inline void rsp_deinterleave_f64(const double* in, size_t n, double* re, double* im) {
    size_t i;
    for (i = 0; i < n; ++i) {
        re[i] = in[2 * i];
        im[i] = in[2 * i + 1];
    }
}
#endif
