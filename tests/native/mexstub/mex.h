/* Declarations of the MATLAB C Matrix / MEX API functions rsp_mex.c uses (both the R2018a
 * interleaved-complex API and the separate-complex one, as documented by MathWorks), for a compile-only syntax check of the gateway in
 * the CPU test suite (tests/test_mex_gateway.py).  Not a MATLAB implementation: nothing links
 * against it. */
#ifndef RSP_TEST_MEX_STUB_H
#define RSP_TEST_MEX_STUB_H
#include <stddef.h>
typedef struct mxArray_tag mxArray;
typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct { double real, imag; } mxComplexDouble;
typedef struct { float real, imag; } mxComplexSingle;
typedef enum { mxUNKNOWN_CLASS = 0, mxDOUBLE_CLASS = 6, mxSINGLE_CLASS = 7 } mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
mxArray* mxGetField(const mxArray* pm, mwIndex index, const char* fieldname);
void mxSetField(mxArray* pm, mwIndex index, const char* fieldname, mxArray* pvalue);
double mxGetScalar(const mxArray* pm);
size_t mxGetNumberOfElements(const mxArray* pm);
size_t mxGetM(const mxArray* pm);
mwSize mxGetNumberOfDimensions(const mxArray* pm);
const mwSize* mxGetDimensions(const mxArray* pm);
int mxIsStruct(const mxArray* pm);
int mxIsChar(const mxArray* pm);
int mxIsDouble(const mxArray* pm);
int mxIsSingle(const mxArray* pm);
int mxIsComplex(const mxArray* pm);
/* The two C Matrix APIs: `mex -R2018a` (interleaved complex, typed accessors) and the separate-
 * complex API (mxGetPr / mxGetPi).  MATLAB's matrix.h sets MX_HAS_INTERLEAVED_COMPLEX by the
 * API the gateway is built for; each API's accessors are declared only in its own mode, so a
 * gateway that mixes them fails to compile (-Werror=implicit-function-declaration). */
#ifdef RSP_MEX_STUB_SEPARATE_COMPLEX
#define MX_HAS_INTERLEAVED_COMPLEX 0
double* mxGetPr(const mxArray* pa);
double* mxGetPi(const mxArray* pa);
void* mxGetData(const mxArray* pa);
void* mxGetImagData(const mxArray* pa);
#else
#define MX_HAS_INTERLEAVED_COMPLEX 1
double* mxGetDoubles(const mxArray* pa);
mxComplexDouble* mxGetComplexDoubles(const mxArray* pa);
mxComplexSingle* mxGetComplexSingles(const mxArray* pa);
#endif
int mxGetString(const mxArray* pm, char* str, mwSize strlen);
mxArray* mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char** fieldnames);
mxArray* mxCreateDoubleScalar(double value);
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity complexFlag);
mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID classid, mxComplexity flag);
void* mxCalloc(mwSize n, mwSize size);
void* mxMalloc(mwSize n);
void* mxRealloc(void* ptr, mwSize size);
void mxFree(void* ptr);
double mxGetNaN(void);
void mexErrMsgIdAndTxt(const char* errorid, const char* errormsg, ...);
int mexAtExit(void (*exit_fcn)(void));
#endif
