/* CPU test of the MEX gateway's separate-complex path (rsp_mx_complex.h built without the
 * interleaved API): a minimal in-memory mxArray stands in for MATLAB's, the conversion helpers
 * run on it, and the interleaved buffers librsp would see are checked element by element
 * (complex double and single inputs, a real array widened, a complex output split back). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"   /* tests/native/mexstub, compiled with -DRSP_MEX_STUB_SEPARATE_COMPLEX */

struct mxArray_tag {
    mxClassID cls;
    int cplx;
    size_t n;
    void* re;
    void* im;
};
double* mxGetPr(const mxArray* a) { return (double*)a->re; }
double* mxGetPi(const mxArray* a) { return (double*)a->im; }
void* mxGetData(const mxArray* a) { return a->re; }
void* mxGetImagData(const mxArray* a) { return a->im; }
size_t mxGetNumberOfElements(const mxArray* a) { return a->n; }
int mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
int mxIsSingle(const mxArray* a) { return a->cls == mxSINGLE_CLASS; }
int mxIsComplex(const mxArray* a) { return a->cplx; }
void* mxMalloc(mwSize n) { return malloc(n); }
void mxFree(void* p) { free(p); }

#include "rsp_mx_complex.h"

static int fails = 0;
#define CHECK(c) do { if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)

int main(void) {
    enum { N = 37 };
    double re[N], im[N], out_re[N], out_im[N];
    float fre[N], fim[N];
    size_t i;
    int32_t dt = -1;
    for (i = 0; i < N; ++i) {
        re[i] = 1.5 * i - 7.0;
        im[i] = -0.25 * i * i;
        fre[i] = (float)(3 * i);
        fim[i] = (float)(-1.0 * i - 0.5);
    }
    {   /* complex double in: interleaved copy */
        mxArray a = {mxDOUBLE_CLASS, 1, N, re, im};
        const double* c = (const double*)rsp_mx_complex_in(&a, &dt);
        CHECK(c != NULL && dt == RSP_C128);
        for (i = 0; i < N; ++i) CHECK(c[2 * i] == re[i] && c[2 * i + 1] == im[i]);
        mxFree((void*)c);
    }
    {   /* complex single in */
        mxArray a = {mxSINGLE_CLASS, 1, N, fre, fim};
        const float* c = (const float*)rsp_mx_complex_in(&a, &dt);
        CHECK(c != NULL && dt == RSP_C64);
        for (i = 0; i < N; ++i) CHECK(c[2 * i] == fre[i] && c[2 * i + 1] == fim[i]);
        mxFree((void*)c);
    }
    {   /* a real array is not complex input */
        mxArray a = {mxDOUBLE_CLASS, 0, N, re, NULL};
        CHECK(rsp_mx_complex_in(&a, &dt) == NULL);
        double w[2 * N];
        rsp_interleave_f64(re, NULL, N, w);   /* the gateway's widening of all-real data */
        for (i = 0; i < N; ++i) CHECK(w[2 * i] == re[i] && w[2 * i + 1] == 0.0);
    }
    {   /* complex output: librsp writes pairs, _done splits them into Pr / Pi */
        mxArray a = {mxDOUBLE_CLASS, 1, N, out_re, out_im};
        double* buf = rsp_mx_complex_out(&a);
        for (i = 0; i < N; ++i) {
            buf[2 * i] = re[i];
            buf[2 * i + 1] = im[i];
        }
        rsp_mx_complex_out_done(&a, buf);
        CHECK(!memcmp(out_re, re, sizeof re) && !memcmp(out_im, im, sizeof im));
    }
    {   /* empty arrays */
        mxArray a = {mxDOUBLE_CLASS, 1, 0, re, im};
        const void* c = rsp_mx_complex_in(&a, &dt);
        CHECK(c != NULL);
        mxFree((void*)c);
    }
    printf(fails ? "FAILED %d\n" : "ok\n", fails);
    return fails != 0;
}
