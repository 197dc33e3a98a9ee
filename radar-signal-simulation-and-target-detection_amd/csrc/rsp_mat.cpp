// rsp_mat.cpp -- MAT-file (Level 5 / "-v7") reader and writer for the frame I/O of the
// reference.
//
// The reference's frames travel as `frame_sim_array_%d.mat`, written by MATLAB's default
// `save` (main_simulate_echoes_with_array.m:226-229 saves `raw_iq_data`,
// main_simulate_echoes_with_array_v2.m:285 saves `raw_iq_data_noise_sample` + `servo_angle`)
// and read back with `load` (debug_simulated_data_processing_v3.m:20-22,
// main_test_with_simulated_data.m:195,208,215).  MATLAB's default is the v7 variant of the
// Level-5 format: every variable is one zlib-compressed (miCOMPRESSED) miMATRIX element.
// This file implements that format natively (no MATLAB, no scipy):
//   - reading: 128-byte header, both byte orders, compressed and plain elements, the
//     small-element tag form, every numeric storage type MATLAB uses to shrink a class
//     (a double array of small integers is stored as miUINT8, ...), real/complex, N-D,
//     char arrays (UTF-8/UTF-16); cell/struct/sparse/object variables are listed and skipped;
//   - writing: double / single arrays (real or complex), char rows, optionally compressed.
// Complex data come out interleaved (re, im) like mxGetComplexDoubles (R2018a API), the
// convention of rsp_process_cube; MAT stores the real and imaginary parts as two blocks.
// v7.3 files are HDF5 and not handled (RSP_ERR_UNSUPPORTED with a message).
#include "rsp.h"

#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

__attribute__((visibility("hidden"))) int rsp_set_error(int code, const char* fmt, ...);   // rsp_plan.cpp

namespace {

enum : uint32_t {
    miINT8 = 1, miUINT8 = 2, miINT16 = 3, miUINT16 = 4, miINT32 = 5, miUINT32 = 6, miSINGLE = 7,
    miDOUBLE = 9, miINT64 = 12, miUINT64 = 13, miMATRIX = 14, miCOMPRESSED = 15, miUTF8 = 16,
    miUTF16 = 17, miUTF32 = 18
};
enum : int {
    mxCELL = 1, mxSTRUCT = 2, mxOBJECT = 3, mxCHAR = 4, mxSPARSE = 5, mxDOUBLE = 6, mxSINGLE = 7,
    mxINT8 = 8, mxUINT8 = 9, mxINT16 = 10, mxUINT16 = 11, mxINT32 = 12, mxUINT32 = 13, mxINT64 = 14,
    mxUINT64 = 15
};

int mi_size(uint32_t t) {
    switch (t) {
        case miINT8: case miUINT8: case miUTF8: return 1;
        case miINT16: case miUINT16: case miUTF16: return 2;
        case miINT32: case miUINT32: case miSINGLE: case miUTF32: return 4;
        case miDOUBLE: case miINT64: case miUINT64: return 8;
        default: return 0;
    }
}

// ---- byte sources: the file itself, or an inflated miCOMPRESSED element ----
struct Source {
    virtual ~Source() {}
    // read exactly n bytes (dst may be null: skip); false on EOF / stream error
    virtual bool read(void* dst, size_t n) = 0;
};

struct FileSource : Source {
    FILE* f;
    explicit FileSource(FILE* f_) : f(f_) {}
    bool read(void* dst, size_t n) override {
        if (!dst) return fseeko(f, (off_t)n, SEEK_CUR) == 0;
        return fread(dst, 1, n, f) == n;
    }
};

// Streaming inflate of `clen` compressed bytes of the file (the element body).
struct ZSource : Source {
    FILE* f;
    size_t remaining_in;
    z_stream zs{};
    std::vector<unsigned char> inbuf;
    bool ok = false, end = false;
    ZSource(FILE* f_, size_t clen) : f(f_), remaining_in(clen), inbuf(1 << 20) {
        ok = inflateInit(&zs) == Z_OK;
    }
    ~ZSource() override { if (ok) inflateEnd(&zs); }
    bool read(void* dst, size_t n) override {
        if (!ok) return false;
        std::vector<unsigned char> scratch;
        unsigned char* out = static_cast<unsigned char*>(dst);
        if (!out) { scratch.resize(std::min<size_t>(n, 1 << 20)); }
        while (n > 0) {
            if (end) return false;
            const size_t chunk = out ? std::min<size_t>(n, 1u << 30) : std::min(n, scratch.size());
            zs.next_out = out ? out : scratch.data();
            zs.avail_out = (uInt)chunk;
            while (zs.avail_out > 0) {
                if (zs.avail_in == 0) {
                    if (remaining_in == 0) return false;
                    const size_t r = std::min(remaining_in, inbuf.size());
                    if (fread(inbuf.data(), 1, r, f) != r) return false;
                    remaining_in -= r;
                    zs.next_in = inbuf.data();
                    zs.avail_in = (uInt)r;
                }
                const int rc = inflate(&zs, Z_NO_FLUSH);
                if (rc == Z_STREAM_END) { end = true; break; }
                if (rc != Z_OK) return false;
            }
            const size_t got = chunk - zs.avail_out;
            if (got != chunk) return false;
            if (out) out += got;
            n -= got;
        }
        return true;
    }
    // consume what is left of the compressed element so the file position is the next element
    bool finish() {
        if (remaining_in) return fseeko(f, (off_t)remaining_in, SEEK_CUR) == 0;
        return true;
    }
};

inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

struct Reader {
    bool swap = false;
    uint32_t u32(uint32_t v) const { return swap ? bswap32(v) : v; }
    void fix(void* p, int sz, size_t n) const {
        if (!swap || sz == 1) return;
        unsigned char* b = static_cast<unsigned char*>(p);
        for (size_t i = 0; i < n; ++i, b += sz)
            for (int j = 0; j < sz / 2; ++j) std::swap(b[j], b[sz - 1 - j]);
    }
    // data element tag; small form (upper half non-zero) carries <= 4 data bytes inline
    bool tag(Source& s, uint32_t& type, uint32_t& nbytes, bool& small, unsigned char inl[4]) const {
        uint32_t w[2];
        if (!s.read(w, 8)) return false;
        const uint32_t t = u32(w[0]);
        if (t >> 16) {
            small = true;
            type = t & 0xFFFF;
            nbytes = t >> 16;
            if (nbytes > 4) return false;   // the small form holds at most 4 bytes inline (malformed file)
            memcpy(inl, &w[1], 4);
        } else {
            small = false;
            type = t;
            nbytes = u32(w[1]);
        }
        return true;
    }
    // a whole sub-element into `buf` (padding consumed)
    bool sub(Source& s, uint32_t& type, std::vector<unsigned char>& buf) const {
        uint32_t nb;
        bool small;
        unsigned char inl[4];
        if (!tag(s, type, nb, small, inl)) return false;
        buf.resize(nb);
        if (small) { memcpy(buf.data(), inl, nb); return true; }
        if (nb && !s.read(buf.data(), nb)) return false;
        const size_t pad = (8 - (nb & 7)) & 7;
        return pad == 0 || s.read(nullptr, pad);
    }
};

struct VarHeader {
    std::string name;
    int cls = 0;
    bool complex = false;
    std::vector<int64_t> dims;
    int64_t numel() const {
        int64_t n = 1;
        for (auto d : dims) n *= d;
        return n;
    }
};

// Convert n stored values of mi type `t` to double.
template <class T>
void conv_from(const unsigned char* src, size_t n, double* dst, size_t stride) {
    for (size_t i = 0; i < n; ++i) {
        T v;
        memcpy(&v, src + i * sizeof(T), sizeof(T));
        dst[i * stride] = (double)v;
    }
}
bool to_double(uint32_t t, const unsigned char* src, size_t n, double* dst, size_t stride) {
    switch (t) {
        case miINT8: conv_from<int8_t>(src, n, dst, stride); return true;
        case miUINT8: conv_from<uint8_t>(src, n, dst, stride); return true;
        case miINT16: conv_from<int16_t>(src, n, dst, stride); return true;
        case miUINT16: conv_from<uint16_t>(src, n, dst, stride); return true;
        case miINT32: conv_from<int32_t>(src, n, dst, stride); return true;
        case miUINT32: conv_from<uint32_t>(src, n, dst, stride); return true;
        case miSINGLE: conv_from<float>(src, n, dst, stride); return true;
        case miDOUBLE: conv_from<double>(src, n, dst, stride); return true;
        case miINT64: conv_from<int64_t>(src, n, dst, stride); return true;
        case miUINT64: conv_from<uint64_t>(src, n, dst, stride); return true;
        default: return false;
    }
}

// What to do with a miMATRIX body after its header: decide() looks at the header and
// points out_* at the destination (or leaves them null to skip the variable).
struct Want {
    std::function<void(const VarHeader&, Want&)> decide;
    double* out_d = nullptr;      // numeric -> double (interleaved complex)
    float* out_f = nullptr;       // numeric -> float (interleaved complex)
    char* out_s = nullptr;        // char -> UTF-8 bytes, NUL terminated
    int64_t cap = 0;              // entries of out_* (complex counts re and im)
    int nread = 0;                // variables read so far
    int rc = RSP_OK;
};

// Stream a numeric part (real or imag) into the caller's buffer through a bounded staging
// vector, so a 300 MB frame never exists twice in host memory.
bool read_part(const Reader& R, Source& s, int64_t numel, bool cplx, int part, Want& w) {
    uint32_t type, nb;
    bool small;
    unsigned char inl[4];
    if (!R.tag(s, type, nb, small, inl)) return false;
    const int sz = mi_size(type);
    if (!sz || nb % sz) return false;
    const size_t n = nb / sz;
    if ((int64_t)n != numel) {
        w.rc = rsp_set_error(RSP_ERR_INVALID, "MAT: %s part holds %zu values, dims say %lld", part ? "imag" : "real", n,
                             (long long)numel);
        return false;
    }
    const size_t stride = cplx ? 2 : 1;
    const size_t per = (size_t)1 << 20;
    std::vector<unsigned char> stage(small ? 4 : std::min(nb ? (size_t)nb : 1, per * sz));
    std::vector<double> tmp;
    size_t done = 0;
    while (done < n) {
        const size_t k = small ? n : std::min(per, n - done);
        if (small) memcpy(stage.data(), inl, nb);
        else if (!s.read(stage.data(), k * sz)) return false;
        R.fix(stage.data(), sz, k);
        if (w.out_d) {
            if (!to_double(type, stage.data(), k, w.out_d + done * stride + part, stride)) return false;
        } else {
            tmp.resize(k);
            if (!to_double(type, stage.data(), k, tmp.data(), 1)) return false;
            float* o = w.out_f + done * stride + part;
            for (size_t i = 0; i < k; ++i) o[i * stride] = (float)tmp[i];
        }
        done += k;
    }
    if (!small) {
        const size_t pad = (8 - (nb & 7)) & 7;
        if (pad && !s.read(nullptr, pad)) return false;
    }
    return true;
}

// Parse a miMATRIX body of `nbytes` from s: fills hdr, asks w.decide where the data go,
// reads them there or skips the body (lazy: a compressed body that is not wanted is never
// inflated, the caller seeks over it).  Returns false on a malformed element.
bool parse_matrix(const Reader& R, Source& s, uint32_t nbytes, bool lazy_skip, VarHeader& hdr, Want& w) {
    std::vector<unsigned char> b;
    uint32_t t;
    size_t used = 0;
    auto subsz = [](size_t nb) { return nb <= 4 ? 8 : 8 + ((nb + 7) & ~(size_t)7); };
    if (nbytes == 0) return true;   // empty placeholder element
    if (!R.sub(s, t, b) || b.size() < 8) return false;
    used += subsz(b.size());
    uint32_t flags;
    memcpy(&flags, b.data(), 4);
    flags = R.u32(flags);
    hdr.cls = flags & 0xFF;
    hdr.complex = (flags >> 11) & 1;   // flags byte (bits 8..15 of the word): complex = 0x08
    if (!R.sub(s, t, b)) return false;
    used += subsz(b.size());
    const int dsz = mi_size(t);
    if (!dsz) return false;
    hdr.dims.clear();
    for (size_t i = 0; i + dsz <= b.size(); i += dsz) {
        int64_t d = 0;
        if (dsz == 4) { int32_t v; memcpy(&v, &b[i], 4); R.fix(&v, 4, 1); d = v; }
        else if (dsz == 8) { int64_t v; memcpy(&v, &b[i], 8); R.fix(&v, 8, 1); d = v; }
        else return false;
        hdr.dims.push_back(d);
    }
    if (!R.sub(s, t, b)) return false;
    used += subsz(b.size());
    hdr.name.assign(reinterpret_cast<const char*>(b.data()), b.size());
    const bool numeric = hdr.cls >= mxDOUBLE && hdr.cls <= mxUINT64;
    w.out_d = nullptr;
    w.out_f = nullptr;
    w.out_s = nullptr;
    w.cap = 0;
    if (w.decide) w.decide(hdr, w);
    auto skip_rest = [&]() { return lazy_skip || nbytes <= used || s.read(nullptr, nbytes - used); };
    if (!w.out_d && !w.out_f && !w.out_s) return skip_rest();
    ++w.nread;
    const int64_t numel = hdr.numel();
    if (numeric && (w.out_d || w.out_f)) {
        const int64_t need = numel * (hdr.complex ? 2 : 1);
        if (need > w.cap) {
            w.rc = rsp_set_error(RSP_ERR_OVERFLOW, "MAT: variable '%s' has %lld values, buffer holds %lld",
                                 hdr.name.c_str(), (long long)need, (long long)w.cap);
            return skip_rest();
        }
        if (!read_part(R, s, numel, hdr.complex, 0, w)) return false;
        if (hdr.complex && !read_part(R, s, numel, true, 1, w)) return false;
        return true;   // a numeric body ends after its parts
    }
    if (hdr.cls == mxCHAR && w.out_s) {
        if (!R.sub(s, t, b)) return false;
        std::string o;
        const int sz = mi_size(t);
        if (!sz) return false;
        for (size_t i = 0; i + sz <= b.size(); i += sz) {
            uint32_t cp = 0;
            if (sz == 1) cp = b[i];
            else if (sz == 2) { uint16_t v; memcpy(&v, &b[i], 2); R.fix(&v, 2, 1); cp = v; }
            else { uint32_t v; memcpy(&v, &b[i], 4); R.fix(&v, 4, 1); cp = v; }
            if (t == miUTF8 || cp < 0x80) o.push_back((char)cp);
            else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
            else if (cp < 0x10000) {
                o.push_back((char)(0xE0 | (cp >> 12)));
                o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
                o.push_back((char)(0x80 | (cp & 0x3F)));
            } else {
                o.push_back((char)(0xF0 | (cp >> 18)));
                o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
                o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
                o.push_back((char)(0x80 | (cp & 0x3F)));
            }
        }
        if ((int64_t)o.size() + 1 > w.cap) {
            w.rc = rsp_set_error(RSP_ERR_OVERFLOW, "MAT: char variable '%s' needs %zu bytes", hdr.name.c_str(),
                                 o.size() + 1);
            return false;
        }
        memcpy(w.out_s, o.c_str(), o.size() + 1);
        used += subsz(b.size());
        return skip_rest();
    }
    w.rc = rsp_set_error(RSP_ERR_UNSUPPORTED, "MAT: variable '%s' has class %d: only numeric and char arrays are read",
                         hdr.name.c_str(), hdr.cls);
    return skip_rest();
}

struct MatFile {
    FILE* f = nullptr;
    Reader R;
    ~MatFile() { if (f) fclose(f); }
    int open(const char* path) {
        if (!path) return rsp_set_error(RSP_ERR_INVALID, "null path");
        f = fopen(path, "rb");
        if (!f) return rsp_set_error(RSP_ERR_INVALID, "cannot open '%s'", path);
        unsigned char h[128];
        if (fread(h, 1, 128, f) != 128) return rsp_set_error(RSP_ERR_INVALID, "'%s': shorter than a MAT header", path);
        if (!memcmp(h, "\x89HDF", 4) || (h[124] == 0 && h[125] == 2))
            return rsp_set_error(RSP_ERR_UNSUPPORTED, "'%s': MAT v7.3 (HDF5) files are not supported; save with -v7", path);
        if (h[126] == 'I' && h[127] == 'M') R.swap = false;
        else if (h[126] == 'M' && h[127] == 'I') R.swap = true;
        else return rsp_set_error(RSP_ERR_INVALID, "'%s': not a MAT Level 5 file", path);
        return RSP_OK;
    }
    // Visit every top-level variable: w.decide routes its data, then cb(hdr) runs; cb
    // returning true stops the scan.
    template <class CB>
    int scan(Want& w, CB cb) {
        for (;;) {
            uint32_t type, nb;
            bool small;
            unsigned char inl[4];
            FileSource fs(f);
            if (!R.tag(fs, type, nb, small, inl)) return RSP_OK;   // clean EOF
            VarHeader hdr;
            bool ok = true;
            if (type == miCOMPRESSED) {
                ZSource zs(f, nb);
                uint32_t it, inb;
                bool ismall;
                unsigned char iinl[4];
                ok = R.tag(zs, it, inb, ismall, iinl) && it == miMATRIX && parse_matrix(R, zs, inb, true, hdr, w) &&
                     zs.finish();
                if (!ok && w.rc == RSP_OK) w.rc = rsp_set_error(RSP_ERR_INVALID, "MAT: corrupt compressed element");
            } else if (type == miMATRIX) {
                const off_t at = ftello(f);
                ok = parse_matrix(R, fs, nb, false, hdr, w);
                // re-sync on the element boundary (the body is 8-byte aligned)
                ok = ok && fseeko(f, at + (off_t)nb + (off_t)((8 - (nb & 7)) & 7), SEEK_SET) == 0;
                if (!ok && w.rc == RSP_OK) w.rc = rsp_set_error(RSP_ERR_INVALID, "MAT: corrupt matrix element");
            } else {
                ok = small || fs.read(nullptr, nb + ((8 - (nb & 7)) & 7));
            }
            if (w.rc != RSP_OK) return w.rc;
            if (!ok) return rsp_set_error(RSP_ERR_INVALID, "MAT: truncated file");
            if ((type == miCOMPRESSED || type == miMATRIX) && cb(hdr)) return RSP_OK;
        }
    }
};

// ---- writer ----
// One zlib stream (what a miCOMPRESSED element holds) deflated by several threads: each
// 4 MiB chunk is an independent raw-deflate run ending on a byte boundary (Z_SYNC_FLUSH;
// the last one Z_FINISH), the runs are concatenated behind the zlib header, and the
// Adler-32 of the whole input is combined from the per-chunk checksums.  A 290 MB frame
// is mostly incompressible noise, which single-threaded deflate crawls through.
bool zlib_parallel(const unsigned char* src, size_t n, std::vector<unsigned char>& out) {
    const size_t chunk = (size_t)4 << 20;
    const size_t nch = std::max<size_t>(1, (n + chunk - 1) / chunk);
    std::vector<std::vector<unsigned char>> parts(nch);
    std::vector<uLong> adl(nch);
    std::atomic<size_t> next{0};
    std::atomic<bool> ok{true};
    auto work = [&]() {
        for (size_t i; (i = next.fetch_add(1)) < nch;) {
            const size_t a = i * chunk, len = std::min(chunk, n - std::min(n, a));
            z_stream zs{};
            if (deflateInit2(&zs, 1, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) { ok = false; return; }
            parts[i].resize(deflateBound(&zs, len) + 16);
            zs.next_in = const_cast<unsigned char*>(src + a);
            zs.avail_in = (uInt)len;
            zs.next_out = parts[i].data();
            zs.avail_out = (uInt)parts[i].size();
            const int rc = deflate(&zs, i + 1 == nch ? Z_FINISH : Z_SYNC_FLUSH);
            if ((i + 1 == nch && rc != Z_STREAM_END) || (i + 1 < nch && rc != Z_OK) || zs.avail_in) ok = false;
            parts[i].resize(zs.total_out);
            deflateEnd(&zs);
            adl[i] = adler32(adler32(0L, Z_NULL, 0), src + a, (uInt)len);
        }
    };
    const unsigned hw = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    const unsigned nt = (unsigned)std::min<size_t>(hw, nch);
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    if (!ok) return false;
    out.clear();
    out.push_back(0x78);   // zlib header: deflate, 32 KiB window, level "fastest"
    out.push_back(0x01);
    uLong ad = adl[0];
    for (size_t i = 0; i < nch; ++i) {
        out.insert(out.end(), parts[i].begin(), parts[i].end());
        if (i) ad = adler32_combine(ad, adl[i], (z_off_t)std::min(chunk, n - i * chunk));
    }
    for (int k = 3; k >= 0; --k) out.push_back((unsigned char)(ad >> (8 * k)));
    return true;
}

struct Writer {
    std::vector<unsigned char> buf;
    void put(const void* p, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(p);
        buf.insert(buf.end(), b, b + n);
    }
    void pad() { while (buf.size() & 7) buf.push_back(0); }
    void tag(uint32_t type, uint32_t nb) { put(&type, 4); put(&nb, 4); }
    void element(uint32_t type, const void* data, size_t nb) {
        if (nb <= 4 && nb > 0) {   // small data element
            const uint32_t t = type | ((uint32_t)nb << 16);
            put(&t, 4);
            unsigned char z[4] = {0, 0, 0, 0};
            memcpy(z, data, nb);
            put(z, 4);
            return;
        }
        tag(type, (uint32_t)nb);
        put(data, nb);
        pad();
    }
};

int write_var(FILE* f, const rsp_mat_wvar& v, bool compress) {
    if (!v.name || !*v.name || strlen(v.name) > 63) return rsp_set_error(RSP_ERR_INVALID, "MAT: bad variable name");
    if (v.ndims < 2 || v.ndims > 32 || !v.dims) return rsp_set_error(RSP_ERR_INVALID, "MAT: '%s' needs 2..32 dims", v.name);
    int64_t n = 1;
    for (int i = 0; i < v.ndims; ++i) {
        if (v.dims[i] < 0 || v.dims[i] > INT32_MAX) return rsp_set_error(RSP_ERR_INVALID, "MAT: bad dims");
        n *= v.dims[i];
    }
    const bool is_char = v.cls == RSP_MAT_CHAR;
    if (!is_char && v.cls != RSP_MAT_DOUBLE && v.cls != RSP_MAT_SINGLE)
        return rsp_set_error(RSP_ERR_UNSUPPORTED, "MAT: writer handles double, single and char");
    if (n && !v.data) return rsp_set_error(RSP_ERR_INVALID, "MAT: '%s' has no data", v.name);
    const int esz = is_char ? 2 : (v.cls == RSP_MAT_DOUBLE ? 8 : 4);
    const uint64_t body = (uint64_t)n * esz * (v.is_complex ? 2 : 1);
    if (body > 0x7FFFFFF0ull) return rsp_set_error(RSP_ERR_UNSUPPORTED, "MAT: '%s' exceeds 2 GB (needs v7.3)", v.name);
    Writer w;
    w.tag(miMATRIX, 0);   // size patched below
    uint32_t fl[2] = {(uint32_t)(is_char ? mxCHAR : (v.cls == RSP_MAT_DOUBLE ? mxDOUBLE : mxSINGLE)) |
                          (v.is_complex && !is_char ? 0x800u : 0u),
                      0};
    w.element(miUINT32, fl, 8);
    std::vector<int32_t> d(v.dims, v.dims + v.ndims);
    w.element(miINT32, d.data(), d.size() * 4);
    w.element(miINT8, v.name, strlen(v.name));
    if (is_char) {
        const unsigned char* s = static_cast<const unsigned char*>(v.data);
        std::vector<uint16_t> u(n);
        for (int64_t i = 0; i < n; ++i) u[i] = s[i];
        w.element(miUTF16, u.data(), u.size() * 2);
    } else {
        const uint32_t t = v.cls == RSP_MAT_DOUBLE ? miDOUBLE : miSINGLE;
        for (int part = 0; part < (v.is_complex ? 2 : 1); ++part) {
            w.tag(t, (uint32_t)(n * esz));
            const size_t at = w.buf.size();
            w.buf.resize(at + (size_t)n * esz);
            unsigned char* o = w.buf.data() + at;
            const unsigned char* src = static_cast<const unsigned char*>(v.data);
            if (!v.is_complex) memcpy(o, src, (size_t)n * esz);
            else
                for (int64_t i = 0; i < n; ++i) memcpy(o + i * esz, src + (2 * i + part) * esz, esz);
            w.pad();
        }
    }
    const uint32_t total = (uint32_t)(w.buf.size() - 8);
    memcpy(w.buf.data() + 4, &total, 4);
    if (!compress) return fwrite(w.buf.data(), 1, w.buf.size(), f) == w.buf.size() ? RSP_OK : rsp_set_error(RSP_ERR_INVALID, "MAT: write failed");
    std::vector<unsigned char> c;
    if (!zlib_parallel(w.buf.data(), w.buf.size(), c)) return rsp_set_error(RSP_ERR_NOMEM, "MAT: zlib compress failed");
    uint32_t hdr[2] = {miCOMPRESSED, (uint32_t)c.size()};
    // MATLAB writes compressed elements unpadded; readers follow the tag's byte count
    if (fwrite(hdr, 4, 2, f) != 2 || fwrite(c.data(), 1, c.size(), f) != c.size())
        return rsp_set_error(RSP_ERR_INVALID, "MAT: write failed");
    return RSP_OK;
}

}  // namespace

extern "C" {

int32_t rsp_mat_list(const char* path, rsp_mat_var* vars, int32_t cap, int32_t* n_vars) {
    if (!n_vars || (cap > 0 && !vars)) return rsp_set_error(RSP_ERR_INVALID, "null argument");
    MatFile m;
    int rc = m.open(path);
    if (rc) return rc;
    Want w;
    int n = 0;
    rc = m.scan(w, [&](const VarHeader& h) {
        if (n < cap) {
            rsp_mat_var& v = vars[n];
            memset(&v, 0, sizeof(v));
            snprintf(v.name, sizeof(v.name), "%s", h.name.c_str());
            v.cls = h.cls;
            v.is_complex = h.complex;
            v.ndims = (int32_t)std::min<size_t>(h.dims.size(), RSP_MAT_MAXDIMS);
            for (int i = 0; i < v.ndims; ++i) v.dims[i] = h.dims[i];
            v.numel = h.numel();
        }
        ++n;
        return false;
    });
    *n_vars = n;
    return rc;
}

int32_t rsp_mat_read(const char* path, const char* name, int32_t dtype, void* out, int64_t cap) {
    if (!name || !out) return rsp_set_error(RSP_ERR_INVALID, "null argument");
    if (dtype != RSP_MAT_OUT_F64 && dtype != RSP_MAT_OUT_F32 && dtype != RSP_MAT_OUT_CHAR)
        return rsp_set_error(RSP_ERR_INVALID, "MAT: unknown output dtype %d", dtype);
    MatFile m;
    int rc = m.open(path);
    if (rc) return rc;
    Want w;
    bool hit = false;
    w.decide = [&](const VarHeader& h, Want& ww) {
        if (h.name != name) return;
        hit = true;
        ww.cap = cap;
        if (dtype == RSP_MAT_OUT_F64) ww.out_d = static_cast<double*>(out);
        else if (dtype == RSP_MAT_OUT_F32) ww.out_f = static_cast<float*>(out);
        else ww.out_s = static_cast<char*>(out);
    };
    rc = m.scan(w, [&](const VarHeader&) { return hit; });
    if (rc) return rc;
    if (!hit) return rsp_set_error(RSP_ERR_INVALID, "MAT: '%s' has no variable '%s'", path, name);
    return RSP_OK;
}

int32_t rsp_mat_write(const char* path, const rsp_mat_wvar* vars, int32_t n, int32_t compress) {
    if (!path || (n > 0 && !vars) || n < 0) return rsp_set_error(RSP_ERR_INVALID, "null argument");
    FILE* f = fopen(path, "wb");
    if (!f) return rsp_set_error(RSP_ERR_INVALID, "cannot create '%s'", path);
    char h[128];
    memset(h, ' ', 116);
    const int k = snprintf(h, 116, "MATLAB 5.0 MAT-file, Platform: GLNXA64, Created by: librsp (rsp_mat_write)");
    if (k > 0 && k < 116) h[k] = ' ';
    memset(h + 116, 0, 8);   // no subsystem data
    h[124] = 0x00;
    h[125] = 0x01;           // version 0x0100, little-endian
    h[126] = 'I';
    h[127] = 'M';
    int rc = RSP_OK;
    if (fwrite(h, 1, 128, f) != 128) rc = rsp_set_error(RSP_ERR_INVALID, "MAT: write failed");
    for (int i = 0; rc == RSP_OK && i < n; ++i) rc = write_var(f, vars[i], compress != 0);
    if (fclose(f) != 0 && rc == RSP_OK) rc = rsp_set_error(RSP_ERR_INVALID, "MAT: close failed");
    return rc;
}

int32_t rsp_mat_load_frame(const char* path, int32_t dtype, void* cube, int64_t cap_elems, int32_t dims_out[3],
                           double* servo_angle, int32_t angle_cap, int32_t* n_angle) {
    if (!path || !dims_out) return rsp_set_error(RSP_ERR_INVALID, "null argument");
    if (dtype != RSP_C64 && dtype != RSP_C128) return rsp_set_error(RSP_ERR_INVALID, "dtype must be RSP_C64/RSP_C128");
    MatFile m;
    int rc = m.open(path);
    if (rc) return rc;
    // the echo cube under either generation's name (v1 main_simulate_echoes_with_array.m:229,
    // v2 main_simulate_echoes_with_array_v2.m:285, loader debug_simulated_data_processing_v3.m:21),
    // read straight into the caller's buffer in one pass over the file
    bool got_cube = false, real_cube = false;
    int64_t numel = 0;
    int na = 0;
    std::vector<double> stage_d;
    std::vector<float> stage_f;
    Want w;
    w.decide = [&](const VarHeader& h, Want& ww) {
        const bool numeric = h.cls >= mxDOUBLE && h.cls <= mxUINT64;
        if ((h.name == "raw_iq_data_noise_sample" || h.name == "raw_iq_data") && !got_cube) {
            if (!numeric || h.dims.size() < 2 || h.dims.size() > 3) {
                ww.rc = rsp_set_error(RSP_ERR_INVALID, "MAT: %s must be a numeric [P x N x C] array", h.name.c_str());
                return;
            }
            got_cube = true;
            numel = h.numel();
            for (int i = 0; i < 3; ++i) dims_out[i] = i < (int)h.dims.size() ? (int32_t)h.dims[i] : 1;
            if (!cube) return;
            if (numel > cap_elems) {
                ww.rc = rsp_set_error(RSP_ERR_OVERFLOW, "MAT: cube has %lld samples, buffer %lld", (long long)numel,
                                      (long long)cap_elems);
                return;
            }
            real_cube = !h.complex;
            // complex: interleaved straight into the caller's buffer; real: staged, widened below
            if (dtype == RSP_C128) {
                if (real_cube) { stage_d.resize(numel); ww.out_d = stage_d.data(); }
                else ww.out_d = static_cast<double*>(cube);
            } else {
                if (real_cube) { stage_f.resize(numel); ww.out_f = stage_f.data(); }
                else ww.out_f = static_cast<float*>(cube);
            }
            ww.cap = numel * (real_cube ? 1 : 2);
        } else if (h.name == "servo_angle" && numeric) {
            na = (int)h.numel();
            if (!servo_angle || angle_cap <= 0) return;
            if (h.complex || na > angle_cap) {
                ww.rc = rsp_set_error(RSP_ERR_OVERFLOW, "MAT: servo_angle has %d values (cap %d)", na, angle_cap);
                return;
            }
            ww.out_d = servo_angle;
            ww.cap = angle_cap;
        }
    };
    rc = m.scan(w, [](const VarHeader&) { return false; });
    if (rc) return rc;
    if (!got_cube) return rsp_set_error(RSP_ERR_INVALID, "MAT: '%s' holds neither raw_iq_data_noise_sample nor raw_iq_data", path);
    if (cube && real_cube) {   // real-valued cube: zero imaginary part
        if (dtype == RSP_C128) {
            double* o = static_cast<double*>(cube);
            for (int64_t i = 0; i < numel; ++i) { o[2 * i] = stage_d[i]; o[2 * i + 1] = 0.0; }
        } else {
            float* o = static_cast<float*>(cube);
            for (int64_t i = 0; i < numel; ++i) { o[2 * i] = stage_f[i]; o[2 * i + 1] = 0.f; }
        }
    }
    if (n_angle) *n_angle = na;
    return RSP_OK;
}

int32_t rsp_mat_save_frame(const char* path, const double* cube, int32_t P, int32_t N, int32_t C,
                           const double* servo_angle, int32_t n_angle, int32_t generation, int32_t compress) {
    if (!path || !cube || P < 1 || N < 1 || C < 1) return rsp_set_error(RSP_ERR_INVALID, "bad argument");
    if (generation != 1 && generation != 2) return rsp_set_error(RSP_ERR_INVALID, "generation must be 1 or 2");
    const int64_t d3[3] = {P, N, C};
    const int64_t da[2] = {1, n_angle};
    rsp_mat_wvar v[2];
    memset(v, 0, sizeof(v));
    v[0].name = generation == 2 ? "raw_iq_data_noise_sample" : "raw_iq_data";
    v[0].cls = RSP_MAT_DOUBLE;
    v[0].is_complex = 1;
    v[0].ndims = 3;
    v[0].dims = d3;
    v[0].data = cube;
    v[1].name = "servo_angle";
    v[1].cls = RSP_MAT_DOUBLE;
    v[1].ndims = 2;
    v[1].dims = da;
    v[1].data = servo_angle;
    return rsp_mat_write(path, v, (servo_angle && n_angle > 0) ? 2 : 1, compress);
}

}  // extern "C"
