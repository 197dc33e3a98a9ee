/* rsp_mx_complex.h -- the MEX gateway's access to numeric data, for both MATLAB C Matrix APIs.
 *
 *   mex -R2018a rsp_mex.c ...   interleaved complex (MX_HAS_INTERLEAVED_COMPLEX = 1): the
 *                               gateway hands MATLAB's own buffers (mxGetComplexDoubles /
 *                               mxGetComplexSingles) to librsp, no copy;
 *   mex rsp_mex.c ...           the separate-complex API of every release (-R2017b, the default
 *   (or -R2017b)                before R2018a, MX_HAS_INTERLEAVED_COMPLEX = 0): inputs are
 *                               interleaved from mxGetPr / mxGetPi (mxGetData / mxGetImagData for
 *                               single) into mxMalloc'd buffers, complex outputs are written
 *                               interleaved and split into the mxArray after the call.
 *
 * Either way librsp sees the interleaved layout of include/rsp.h.  Buffers made here are
 * mxMalloc'd and freed by MATLAB at the end of the MEX call. */
#ifndef RSP_MX_COMPLEX_H
#define RSP_MX_COMPLEX_H
#include <stdint.h>
#include "mex.h"
#include "rsp.h"
#include "rsp_cplx_pack.h"

#ifndef MX_HAS_INTERLEAVED_COMPLEX
#define MX_HAS_INTERLEAVED_COMPLEX 0
#endif

#if MX_HAS_INTERLEAVED_COMPLEX
static inline double* rsp_mx_doubles(const mxArray* a) { return mxGetDoubles(a); }
/* complex double / single data as interleaved pairs (*dtype RSP_C128 / RSP_C64), or NULL when a
 * is not a complex floating array */
static inline const void* rsp_mx_complex_in(const mxArray* a, int32_t* dtype) {
    if (mxIsDouble(a) && mxIsComplex(a)) { *dtype = RSP_C128; return mxGetComplexDoubles(a); }
    if (mxIsSingle(a) && mxIsComplex(a)) { *dtype = RSP_C64; return mxGetComplexSingles(a); }
    return NULL;
}
/* where librsp writes a complex double output array's interleaved pairs */
static inline double* rsp_mx_complex_out(mxArray* a) { return (double*)mxGetComplexDoubles(a); }
/* after the librsp call: nothing to move with the interleaved API */
static inline void rsp_mx_complex_out_done(mxArray* a, double* buf) { (void)a; (void)buf; }
#else
static inline double* rsp_mx_doubles(const mxArray* a) { return mxGetPr(a); }
static inline const void* rsp_mx_complex_in(const mxArray* a, int32_t* dtype) {
    const size_t n = mxGetNumberOfElements(a);
    if (mxIsDouble(a) && mxIsComplex(a)) {
        double* c = (double*)mxMalloc(2 * (n > 0 ? n : 1) * sizeof(double));
        rsp_interleave_f64(mxGetPr(a), mxGetPi(a), n, c);
        *dtype = RSP_C128;
        return c;
    }
    if (mxIsSingle(a) && mxIsComplex(a)) {
        float* c = (float*)mxMalloc(2 * (n > 0 ? n : 1) * sizeof(float));
        rsp_interleave_f32((const float*)mxGetData(a), (const float*)mxGetImagData(a), n, c);
        *dtype = RSP_C64;
        return c;
    }
    return NULL;
}
static inline double* rsp_mx_complex_out(mxArray* a) {
    const size_t n = mxGetNumberOfElements(a);
    return (double*)mxMalloc(2 * (n > 0 ? n : 1) * sizeof(double));
}
static inline void rsp_mx_complex_out_done(mxArray* a, double* buf) {
    rsp_deinterleave_f64(buf, mxGetNumberOfElements(a), mxGetPr(a), mxGetPi(a));
    mxFree(buf);
}
#endif
#endif
