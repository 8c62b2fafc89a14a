// Host-side native runtime for alink_amd (C ABI, loaded with ctypes).
//
//  * CSV line parsing with Alink CsvParser semantics (A/operator/common/io/csv/CsvParser.java): quoting only
//    for string columns, doubled quote = literal quote, blank non-string token = NULL.  Numeric columns are
//    parsed straight into typed arrays in parallel (OpenMP) — the reference parses row-by-row in Java.
//  * Guava-compatible murmur3_32(seed 0) over UTF-16 code units ("hashUnencodedChars"), used by
//    FeatureHasher (A/operator/common/feature/FeatureHasherMapper.java:37,63-106).
//  * dense vector string parsing ("1 2 3" / "1,2,3") into a row-major double matrix.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>

extern "C" {

// types: 0 = string, 1 = double, 2 = int64, 3 = bool
// out_num[c]: double* (type 1) or int64_t* (types 2, 3) with nlines entries (may be null for string cols)
// out_null[c]: uint8_t* nlines (1 = NULL)
// out_soff[c]: int64_t* 2*nlines (start, end byte offsets into buf; -1 = NULL), for string columns
// out_sesc[c]: uint8_t* nlines (1 = contains escaped quotes to collapse)
// returns -1 - line on parse error, else 0
// alink_csv_parse_spans: the same over lines [line_start[i], line_end[i]) of one buffer (a file read whole, the
// row delimiters left in place between the spans).
int alink_csv_parse_spans(const char* buf, const int64_t* line_off, const int64_t* line_end, int64_t nlines,
                          int ncols, const int* types, char delim, int quote, void** out_num, uint8_t** out_null,
                          int64_t** out_soff, uint8_t** out_sesc) {
    int64_t err = -1;
#pragma omp parallel for schedule(static) if (nlines > 256)
    for (int64_t li = 0; li < nlines; ++li) {
        const char* s = buf + line_off[li];
        const int64_t n = line_end[li] - line_off[li];
        int64_t pos = 0;
        bool ok = true;
        for (int c = 0; c < ncols; ++c) {
            out_null[c][li] = 1;
            if (types[c] == 0) {
                out_soff[c][2 * li] = -1;
                out_soff[c][2 * li + 1] = -1;
                out_sesc[c][li] = 0;
            }
            if (pos > n) {
                if (n != 0) ok = false;  // an empty line (skipBlankLine off) is a row of nulls
                continue;
            }
            // find the end of this field
            int64_t end;
            if (types[c] == 0 && quote >= 0 && pos < n && s[pos] == (char)quote) {
                int64_t p = pos + 1;
                bool esc = false;
                while (p < n) {
                    if (s[p] == (char)quote) {
                        if (!esc) {
                            if (p + 1 < n && s[p + 1] == (char)quote) esc = true;
                            else break;
                        } else {
                            esc = false;
                        }
                    }
                    ++p;
                }
                if (p >= n) end = n;
                else {
                    const char* d = (const char*)memchr(s + p + 1, delim, n - p - 1);
                    end = d ? (d - s) : n;
                }
            } else {
                const char* d = (pos < n) ? (const char*)memchr(s + pos, delim, n - pos) : nullptr;
                end = d ? (d - s) : n;
            }
            const int64_t tl = end - pos;
            if (tl > 0) {
                const char* tok = s + pos;
                if (types[c] == 0) {
                    int64_t a = line_off[li] + pos, b = line_off[li] + end;
                    if (quote >= 0 && tok[0] == (char)quote) {
                        a += 1;
                        if (tl > 1 && tok[tl - 1] == (char)quote) b -= 1;
                        for (int64_t q = 1; q + 1 < tl; ++q)
                            if (tok[q] == (char)quote && tok[q + 1] == (char)quote) { out_sesc[c][li] = 1; break; }
                    }
                    out_soff[c][2 * li] = a;
                    out_soff[c][2 * li + 1] = b;
                    out_null[c][li] = 0;
                } else {
                    int64_t a = 0, b = tl;
                    while (a < b && (tok[a] == ' ' || tok[a] == '\t' || tok[a] == '\r')) ++a;
                    while (b > a && (tok[b - 1] == ' ' || tok[b - 1] == '\t' || tok[b - 1] == '\r')) --b;
                    if (b > a) {
                        std::string t(tok + a, b - a);
                        char* ep = nullptr;
                        if (types[c] == 1) {
                            double v = strtod(t.c_str(), &ep);
                            if (*ep != 0) ok = false;
                            ((double*)out_num[c])[li] = v;
                        } else if (types[c] == 2) {
                            long long v = strtoll(t.c_str(), &ep, 10);
                            if (*ep != 0) {  // allow "3.0"-style integers like Long.parseLong would not; reject
                                ok = false;
                            }
                            ((int64_t*)out_num[c])[li] = (int64_t)v;
                        } else {
                            bool v;
                            if (t == "true" || t == "TRUE" || t == "True" || t == "1") v = true;
                            else if (t == "false" || t == "FALSE" || t == "False" || t == "0") v = false;
                            else { ok = false; v = false; }
                            ((int64_t*)out_num[c])[li] = v ? 1 : 0;
                        }
                        out_null[c][li] = 0;
                    }
                }
            }
            pos = end + 1;
        }
        if (!ok) {
#pragma omp critical
            { if (err < 0 || li < err) err = li; }
        }
    }
    return err >= 0 ? (int)(-1 - err) : 0;
}

int alink_csv_parse(const char* buf, const int64_t* line_off, int64_t nlines, int ncols, const int* types,
                    char delim, int quote, void** out_num, uint8_t** out_null, int64_t** out_soff,
                    uint8_t** out_sesc) {
    return alink_csv_parse_spans(buf, line_off, line_off + 1, nlines, ncols, types, delim, quote, out_num, out_null,
                                 out_soff, out_sesc);
}

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

static inline uint32_t mix_k1(uint32_t k1) {
    k1 *= 0xcc9e2d51u;
    k1 = rotl32(k1, 15);
    k1 *= 0x1b873593u;
    return k1;
}

static inline uint32_t mix_h1(uint32_t h1, uint32_t k1) {
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    h1 = h1 * 5 + 0xe6546b64u;
    return h1;
}

static inline uint32_t fmix(uint32_t h1, uint32_t length) {
    h1 ^= length;
    h1 ^= h1 >> 16;
    h1 *= 0x85ebca6bu;
    h1 ^= h1 >> 13;
    h1 *= 0xc2b2ae35u;
    h1 ^= h1 >> 16;
    return h1;
}

// Guava Murmur3_32HashFunction.hashUnencodedChars(seed) over UTF-16 code units
static int32_t murmur3_utf16(const uint16_t* chars, int64_t len, uint32_t seed) {
    uint32_t h1 = seed;
    int64_t i = 1;
    for (; i < len; i += 2) {
        uint32_t k1 = (uint32_t)chars[i - 1] | ((uint32_t)chars[i] << 16);
        k1 = mix_k1(k1);
        h1 = mix_h1(h1, k1);
    }
    if ((len & 1) == 1) {
        uint32_t k1 = chars[len - 1];
        k1 = mix_k1(k1);
        h1 ^= k1;
    }
    return (int32_t)fmix(h1, (uint32_t)(2 * len));
}

// batch: strings given as UTF-16 code units concatenated, offsets (in code units) n+1
void alink_murmur3_utf16_batch(const uint16_t* chars, const int64_t* off, int64_t n, uint32_t seed,
                               int32_t* out) {
#pragma omp parallel for schedule(static) if (n > 4096)
    for (int64_t i = 0; i < n; ++i) out[i] = murmur3_utf16(chars + off[i], off[i + 1] - off[i], seed);
}

// MurmurHash3_x86_32(seed) over raw bytes (Guava murmur3_32().hashBytes) for n packed strings (bytes, off[n+1])
void alink_murmur3_bytes_batch(const uint8_t* bytes, const int64_t* off, int64_t n, uint32_t seed, int32_t* out) {
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t s = 0; s < n; ++s) {
        const uint8_t* p = bytes + off[s];
        const int64_t len = off[s + 1] - off[s];
        uint32_t h1 = seed;
        const int64_t nb = len >> 2;
        for (int64_t i = 0; i < nb; ++i) {
            uint32_t k;
            std::memcpy(&k, p + 4 * i, 4);
            h1 = mix_h1(h1, mix_k1(k));
        }
        uint32_t k1 = 0;
        const uint8_t* t = p + 4 * nb;
        switch (len & 3) {
            case 3: k1 ^= (uint32_t)t[2] << 16; [[fallthrough]];
            case 2: k1 ^= (uint32_t)t[1] << 8; [[fallthrough]];
            case 1: k1 ^= t[0]; h1 ^= mix_k1(k1);
        }
        out[s] = (int32_t)fmix(h1, (uint32_t)len);
    }
}

// Guava hashUnencodedChars(seed) of prefix (UTF-16 units) ++ the packed UTF-8 strings, decoded to UTF-16 units
// on the fly (the host twin of the HIP murmur3_utf8_index_kernel)
void alink_murmur3_utf8_batch(const uint8_t* bytes, const int64_t* off, int64_t n, const uint16_t* prefix, int plen,
                              uint32_t seed, int32_t* out) {
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t s = 0; s < n; ++s) {
        uint32_t h1 = seed, pending = 0;
        int64_t cnt = 0;
        auto push = [&](uint32_t u) {
            if (cnt & 1) h1 = mix_h1(h1, mix_k1(pending | (u << 16)));
            else pending = u;
            ++cnt;
        };
        for (int j = 0; j < plen; ++j) push(prefix[j]);
        const uint8_t* p = bytes + off[s];
        const int64_t len = off[s + 1] - off[s];
        for (int64_t i = 0; i < len;) {
            const uint32_t b0 = p[i];
            uint32_t cp;
            if (b0 < 0x80u) { cp = b0; i += 1; }
            else if (b0 < 0xE0u && i + 1 < len) { cp = ((b0 & 0x1Fu) << 6) | (p[i + 1] & 0x3Fu); i += 2; }
            else if (b0 < 0xF0u && i + 2 < len) {
                cp = ((b0 & 0x0Fu) << 12) | ((p[i + 1] & 0x3Fu) << 6) | (p[i + 2] & 0x3Fu); i += 3;
            } else if (i + 3 < len) {
                cp = ((b0 & 0x07u) << 18) | ((p[i + 1] & 0x3Fu) << 12) | ((p[i + 2] & 0x3Fu) << 6) | (p[i + 3] & 0x3Fu);
                i += 4;
            } else { cp = 0xFFFDu; i += 1; }
            if (cp >= 0x10000u) {
                const uint32_t c = cp - 0x10000u;
                push(0xD800u + (c >> 10));
                push(0xDC00u + (c & 0x3FFu));
            } else {
                push(cp);
            }
        }
        if (cnt & 1) h1 ^= mix_k1(pending);
        out[s] = (int32_t)fmix(h1, (uint32_t)(2 * cnt));
    }
}

// dense vector strings -> row-major [n][d] doubles (missing tail = 0); returns -1 - row on error
int alink_parse_dense_vectors(const char* buf, const int64_t* off, int64_t n, int64_t d, double* out,
                              int64_t* counts) {
    int64_t err = -1;
#pragma omp parallel for schedule(static) if (n > 64)
    for (int64_t i = 0; i < n; ++i) {
        const char* p = buf + off[i];
        const char* e = buf + off[i + 1];
        double* row = out + i * d;
        for (int64_t j = 0; j < d; ++j) row[j] = 0.0;
        int64_t j = 0;
        std::string tmp;
        while (p < e) {
            while (p < e && (*p == ' ' || *p == ',')) ++p;
            if (p >= e) break;
            const char* q = p;
            while (q < e && *q != ' ' && *q != ',') ++q;
            tmp.assign(p, q - p);
            // plain decimal tokens only: strtod would also take inf / nan / hex forms Double.parseDouble rejects
            // (the caller parses anything else on its general path)
            bool plain = true;
            for (const char* c = p; c < q; ++c)
                plain &= (*c >= '0' && *c <= '9') || *c == '.' || *c == 'e' || *c == 'E' || *c == '+' || *c == '-';
            char* ep = nullptr;
            double v = strtod(tmp.c_str(), &ep);
            if (!plain || *ep != 0 || j >= d) {
#pragma omp critical
                { if (err < 0 || i < err) err = i; }
                break;
            }
            row[j++] = v;
            p = q;
        }
        if (counts != nullptr) counts[i] = j;
    }
    return err >= 0 ? (int)(-1 - err) : 0;
}

// Binary prediction-detail strings {"<label>":p,"<label>":p} (the predictors' detail column, parsed per row by
// BinaryClassMetrics / EvalBinaryClassBatchOp): probability of key0 and key1 for each of n strings.  Returns 0, or
// the 1-based index of the first string it cannot read (not exactly two plain "key":number entries, an escape in a
// key, a missing key), in which case the caller parses with the general JSON reader.
static inline const char* skip_ws(const char* p, const char* e) {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    return p;
}

int64_t alink_parse_binary_detail(const char* buf, const int64_t* off, int64_t n, const char* key0, int len0,
                                  const char* key1, int len1, double* p0, double* p1) {
    for (int64_t i = 0; i < n; ++i) {
        const char* p = buf + off[i];
        const char* e = buf + off[i + 1];
        bool got0 = false, got1 = false;
        int entries = 0;
        p = skip_ws(p, e);
        if (p >= e || *p != '{') return i + 1;
        ++p;
        while (true) {
            p = skip_ws(p, e);
            if (p >= e || *p != '"') return i + 1;
            const char* ks = ++p;
            while (p < e && *p != '"') {
                if (*p == '\\') return i + 1;
                ++p;
            }
            if (p >= e) return i + 1;
            const int klen = (int)(p - ks);
            ++p;
            p = skip_ws(p, e);
            if (p >= e || *p != ':') return i + 1;
            p = skip_ws(p + 1, e);
            char num[64];
            int nl = 0;
            // a number, or a number in a JSON string (HashMap<String,String> details: {"1":"0.3",...})
            const bool quoted = p < e && *p == '"';
            if (quoted) {
                ++p;
                while (p < e && nl < 63 && *p != '"') num[nl++] = *p++;
                if (p >= e || *p != '"') return i + 1;
                ++p;
            } else {
                while (p < e && nl < 63 && *p != ',' && *p != '}' && *p != ' ') num[nl++] = *p++;
            }
            num[nl] = 0;
            char* endp = nullptr;
            const double v = strtod(num, &endp);
            if (nl == 0 || endp != num + nl) return i + 1;
            if (klen == len0 && memcmp(ks, key0, len0) == 0) {
                p0[i] = v;
                got0 = true;
            } else if (klen == len1 && memcmp(ks, key1, len1) == 0) {
                p1[i] = v;
                got1 = true;
            }
            ++entries;
            p = skip_ws(p, e);
            if (p < e && *p == ',') {
                ++p;
                continue;
            }
            if (p < e && *p == '}') break;
            return i + 1;
        }
        if (entries != 2 || !got0 || !got1) return i + 1;
    }
    return 0;
}

int alink_native_version() { return 1; }

}  // extern "C"

// ---------------------------------------------------------------------------------------------------------------
// java.lang.Double.toString for arrays (model snapshots: 1e6 FTRL coefficients, GLM / linear model vectors).
// Digits are the shortest round-trip decimal (std::to_chars, the digits Python's repr gives the reference
// formatter common/javafmt.py:java_double_str); layout per the JVM rules: plain decimal with at least one
// fractional digit for |x| in [1e-3, 1e7), else d.dddE<n>.  Writes "v0,v1,...,vn-1" (no brackets) into out
// (capacity >= 26 * n) and returns the length.
// ---------------------------------------------------------------------------------------------------------------
#include <charconv>
#include <vector>
#include <cmath>
#include <cstring>

// T = float: java.lang.Float.toString -- the same layout over the shortest float32 round-trip digits
template <typename T>
static int java_num_to(T x, char* out) {
    if (std::isnan(x)) { std::memcpy(out, "NaN", 3); return 3; }
    if (std::isinf(x)) {
        if (x > 0) { std::memcpy(out, "Infinity", 8); return 8; }
        std::memcpy(out, "-Infinity", 9); return 9;
    }
    int p = 0;
    if (x == 0.0) {
        if (std::signbit(x)) out[p++] = '-';
        std::memcpy(out + p, "0.0", 3);
        return p + 3;
    }
    if (x < 0) out[p++] = '-';
    const T ax = std::fabs(x);
    char buf[40];
    const auto res = std::to_chars(buf, buf + sizeof(buf), ax, std::chars_format::scientific);
    const char* e = static_cast<const char*>(std::memchr(buf, 'e', (size_t)(res.ptr - buf)));
    char digits[24];
    int nd = 0;
    digits[nd++] = buf[0];
    for (const char* c = buf + 2; c < e; ++c) digits[nd++] = *c;     // after "d."
    while (nd > 1 && digits[nd - 1] == '0') --nd;
    int ex = 0;
    {
        const char* c = e + 1;
        bool neg = false;
        if (*c == '-') { neg = true; ++c; } else if (*c == '+') { ++c; }
        for (; c < res.ptr; ++c) ex = ex * 10 + (*c - '0');
        if (neg) ex = -ex;
    }
    const int point = ex + 1;   // value = 0.digits * 10^point
    if (ax >= 1e-3 && ax < 1e7) {
        if (point <= 0) {
            out[p++] = '0'; out[p++] = '.';
            for (int i = 0; i < -point; ++i) out[p++] = '0';
            for (int i = 0; i < nd; ++i) out[p++] = digits[i];
        } else if (point >= nd) {
            for (int i = 0; i < nd; ++i) out[p++] = digits[i];
            for (int i = nd; i < point; ++i) out[p++] = '0';
            out[p++] = '.'; out[p++] = '0';
        } else {
            for (int i = 0; i < point; ++i) out[p++] = digits[i];
            out[p++] = '.';
            for (int i = point; i < nd; ++i) out[p++] = digits[i];
        }
        return p;
    }
    out[p++] = digits[0];
    out[p++] = '.';
    if (nd > 1) for (int i = 1; i < nd; ++i) out[p++] = digits[i];
    else out[p++] = '0';
    out[p++] = 'E';
    const auto r2 = std::to_chars(out + p, out + p + 8, ex);
    return (int)(r2.ptr - out);
}

static int java_double_to(double x, char* out) { return java_num_to<double>(x, out); }

// n rows of k values: row i = java_double(x[i*k]) sep ... sep java_double(x[i*k+k-1]), rows written back to back;
// row_end[i] = end offset of row i in out (dense-vector strings of a prediction detail column, VectorUtil.toString)
// Large inputs: OpenMP row blocks format into their own slices of out (capacity 26 per value, the bound each
// block is given), then the blocks are compacted left in order.
template <typename T>
static int64_t java_rows(const T* x, int64_t n, int64_t k, char sep, char* out, int64_t* row_end) {
    if (n * k < (1 << 16)) {
        int64_t p = 0;
        for (int64_t i = 0; i < n; ++i) {
            for (int64_t j = 0; j < k; ++j) {
                if (j) out[p++] = sep;
                p += java_num_to<T>(x[i * k + j], out + p);
            }
            row_end[i] = p;
        }
        return p;
    }
    const int64_t rows_per = std::max<int64_t>(1, 8192 / std::max<int64_t>(k, 1));
    const int64_t nb = (n + rows_per - 1) / rows_per;
    std::vector<int64_t> blen(nb);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t r0 = b * rows_per, r1 = std::min(n, r0 + rows_per);
        char* base = out + r0 * k * 26;
        int64_t p = 0;
        for (int64_t i = r0; i < r1; ++i) {
            for (int64_t j = 0; j < k; ++j) {
                if (j) base[p++] = sep;
                p += java_num_to<T>(x[i * k + j], base + p);
            }
            row_end[i] = p;                     // block-relative for now
        }
        blen[b] = p;
    }
    int64_t p = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t r0 = b * rows_per, r1 = std::min(n, r0 + rows_per);
        if (p != r0 * k * 26) std::memmove(out + p, out + r0 * k * 26, (size_t)blen[b]);
        for (int64_t i = r0; i < r1; ++i) row_end[i] += p;
        p += blen[b];
    }
    return p;
}

extern "C" int64_t alink_java_double_rows(const double* x, int64_t n, int64_t k, char sep, char* out,
                                          int64_t* row_end) {
    return java_rows<double>(x, n, k, sep, out, row_end);
}

// n rows of k (int64 key, float32 value) pairs: row i = "key:Float.toString(v),key:v,..." (kvsep ':' and sep ','
// as given) -- the "item:score,..." lists of ALS recommendations.  OpenMP row blocks write into their own
// 48-bytes-per-pair slices of out, then the blocks are compacted in order; row_end[i] = end offset of row i.
extern "C" int64_t alink_java_float_kv_rows(const int64_t* keys, const float* vals, int64_t n, int64_t k,
                                            char kvsep, char sep, char* out, int64_t* row_end) {
    const int64_t W = 48;
    const int64_t rows_per = std::max<int64_t>(1, 8192 / std::max<int64_t>(k, 1));
    const int64_t nb = (n + rows_per - 1) / rows_per;
    std::vector<int64_t> blen(nb);
#pragma omp parallel for schedule(dynamic, 4) if (n * k >= (1 << 16))
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t r0 = b * rows_per, r1 = std::min(n, r0 + rows_per);
        char* base = out + r0 * k * W;
        int64_t p = 0;
        for (int64_t i = r0; i < r1; ++i) {
            for (int64_t j = 0; j < k; ++j) {
                if (j) base[p++] = sep;
                const auto r = std::to_chars(base + p, base + p + 21, keys[i * k + j]);
                p = r.ptr - base;
                base[p++] = kvsep;
                p += java_num_to<float>(vals[i * k + j], base + p);
            }
            row_end[i] = p;
        }
        blen[b] = p;
    }
    int64_t p = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t r0 = b * rows_per, r1 = std::min(n, r0 + rows_per);
        if (p != r0 * k * W) std::memmove(out + p, out + r0 * k * W, (size_t)blen[b]);
        for (int64_t i = r0; i < r1; ++i) row_end[i] += p;
        p += blen[b];
    }
    return p;
}

// the same rows of float32 values in java.lang.Float.toString form (ALS factor strings)
extern "C" int64_t alink_java_float_rows(const float* x, int64_t n, int64_t k, char sep, char* out,
                                         int64_t* row_end) {
    return java_rows<float>(x, n, k, sep, out, row_end);
}

// Threshold sampling of a binary-classification curve over descending thresholds: index 0, then every index
// whose threshold is at least `step` below the last kept one, or within `err` of 0.5 (one sequential scan).
extern "C" int64_t alink_sample_thresholds(const double* thr, int64_t n, double step, double err, int64_t* keep) {
    if (n <= 0) return 0;
    int64_t m = 0;
    keep[m++] = 0;
    double pre = thr[0];
    for (int64_t i = 1; i < n; ++i) {
        if (std::fabs(pre - thr[i]) >= step || std::fabs(thr[i] - 0.5) < err) {
            keep[m++] = i;
            pre = thr[i];
        }
    }
    return m;
}

// Binary evaluation summary of one block (EvalBinaryClass*; reference BinaryMetricsSummary bins): rows with
// code[i] 0 (positive) / 1 (negative) and ok[i] != 0 add to bin floor(p0 * B) (p0 == 1 -> B - 1) of the positive /
// negative half of bins[2B], and -log(clip(p_label, eps, 1 - eps)) to the log loss in row order.
// out2 = {log loss, kept rows}.
extern "C" void alink_binary_bins(const double* probs, int64_t n, int K, int c0, int c1, const int64_t* code,
                                  const uint8_t* ok, int B, double eps, int64_t* bins, double* out2) {
    double ll = 0.0;
    int64_t keep = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t c = code[i];
        if (c < 0 || (ok && !ok[i])) continue;
        const double p0 = probs[i * K + c0];
        const double pl = c == 0 ? p0 : probs[i * K + c1];
        ll += -std::log(std::min(std::max(pl, eps), 1.0 - eps));
        ++keep;
        const double f = p0 == 1.0 ? (double)(B - 1) : std::floor(p0 * B);
        if (f >= 0.0 && f < (double)B) ++bins[(c == 0 ? 0 : B) + (int64_t)f];
    }
    out2[0] = ll;
    out2[1] = (double)keep;
}

extern "C" int64_t alink_java_double_join(const double* x, int64_t n, char* out) {
    // ~90 ns per value on one thread (1e6 coefficients ~0.1 s).  Large inputs are formatted in contiguous chunks,
    // each into its own region of `out` sized for the worst case (26 bytes per value), in parallel, then the chunks
    // are moved down in order; below 2^16 values one thread is faster than the fork / join.
    constexpr int64_t kPar = 1 << 16;
    if (n < kPar) {
        int64_t p = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (i) out[p++] = ',';
            p += java_double_to(x[i], out + p);
        }
        return p;
    }
    const int64_t nch = 64;
    const int64_t per = (n + nch - 1) / nch;
    std::vector<int64_t> len((size_t)nch, 0);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t c = 0; c < nch; ++c) {
        const int64_t a = c * per, b = a + per < n ? a + per : n;
        char* o = out + a * 26;                // chunk c's worst-case region starts at value a's worst-case offset
        int64_t p = 0;
        for (int64_t i = a; i < b; ++i) {
            if (i) o[p++] = ',';
            p += java_double_to(x[i], o + p);
        }
        len[(size_t)c] = p;
    }
    int64_t p = 0;
    for (int64_t c = 0; c < nch; ++c) {      // in order: chunk c's text only moves down (p <= c * per * 26)
        const int64_t a = c * per;
        if (a >= n) break;
        if (p != a * 26) std::memmove(out + p, out + a * 26, (size_t)len[(size_t)c]);
        p += len[(size_t)c];
    }
    return p;
}

// ---------------------------------------------------------------------------------------------------------------
// KV strings ("k1:v1,k2:v2,...": KvToColumns / FormatTrans KV -> COLUMNS with DOUBLE columns) parsed into an
// [n, k] double matrix for the k schema keys.  A line takes the fast path only in its plain form: every field
// non-empty with exactly one value delimiter, and every value of a schema key a plain decimal token (digits, sign,
// '.', exponent; strtod consumes it whole).  flags[i]: bit 0 = the line is not plain (the caller re-parses the
// batch on its general path), bit 1 = a schema key occurs twice (later value kept).  found[i*k + j] = key j seen.
// ---------------------------------------------------------------------------------------------------------------
#include <string_view>
#include <unordered_map>

extern "C" int64_t alink_kv_parse(const char* buf, const int64_t* off, int64_t n, char cd, char vd,
                                  const char* keys, const int64_t* koff, int64_t k, double* out, uint8_t* found,
                                  uint8_t* flags) {
    std::unordered_map<std::string_view, int64_t> pos;
    pos.reserve((size_t)k * 2 + 1);
    for (int64_t j = 0; j < k; ++j) pos.emplace(std::string_view(keys + koff[j], (size_t)(koff[j + 1] - koff[j])), j);
    int64_t nbad = 0;
#pragma omp parallel for schedule(static) reduction(+ : nbad)
    for (int64_t i = 0; i < n; ++i) {
        const char* p = buf + off[i];
        const char* e = buf + off[i + 1];
        double* row = out + i * k;
        uint8_t* fr = found + i * k;
        for (int64_t j = 0; j < k; ++j) {
            row[j] = 0.0;
            fr[j] = 0;
        }
        uint8_t fl = 0;
        char tmp[64];
        if (p == e) fl |= 1;
        while (p < e && !(fl & 1)) {
            const char* q = p;
            while (q < e && *q != cd) ++q;                 // field [p, q)
            const char* d = nullptr;
            int nvd = 0;
            for (const char* c = p; c < q; ++c)
                if (*c == vd) {
                    if (!d) d = c;
                    ++nvd;
                }
            if (q == p || nvd != 1) {
                fl |= 1;
                break;
            }
            auto it = pos.find(std::string_view(p, (size_t)(d - p)));
            if (it != pos.end()) {
                const char* vs = d + 1;
                const int64_t len = q - vs;
                bool plain = len > 0 && len < 63;
                for (const char* c = vs; plain && c < q; ++c)
                    plain = (*c >= '0' && *c <= '9') || *c == '.' || *c == 'e' || *c == 'E' || *c == '+' || *c == '-';
                if (!plain) {
                    fl |= 1;
                    break;
                }
                std::memcpy(tmp, vs, (size_t)len);
                tmp[len] = 0;
                char* ep = nullptr;
                const double v = strtod(tmp, &ep);
                if (*ep != 0) {
                    fl |= 1;
                    break;
                }
                const int64_t j = it->second;
                if (fr[j]) fl |= 2;
                fr[j] = 1;
                row[j] = v;
            }
            p = q < e ? q + 1 : q;
            if (q < e && p == e) fl |= 1;                   // trailing delimiter: an empty last field
        }
        flags[i] = fl;
        nbad += (fl & 1) ? 1 : 0;
    }
    return nbad;
}

// Flat JSON objects ({"k": number, ...}: JsonToColumns / FormatTrans JSON -> COLUMNS with DOUBLE columns) into an
// [n, k] double matrix for the k schema keys.  Plain form only: one object per line, keys plain strings (no
// escapes), every member value a JSON number (members whose key is not in the schema may also be strings without
// escapes); anything else sets flags bit 0 (the caller parses the batch with the general JSON reader).  Integer
// tokens give +0.0 for -0 (the reader turns them into integers first).  A key given twice keeps the later value.
static inline const char* json_ws(const char* p, const char* e) {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    return p;
}

extern "C" int64_t alink_json_flat_parse(const char* buf, const int64_t* off, int64_t n, const char* keys,
                                         const int64_t* koff, int64_t k, double* out, uint8_t* found,
                                         uint8_t* flags) {
    std::unordered_map<std::string_view, int64_t> pos;
    pos.reserve((size_t)k * 2 + 1);
    for (int64_t j = 0; j < k; ++j) pos.emplace(std::string_view(keys + koff[j], (size_t)(koff[j + 1] - koff[j])), j);
    int64_t nbad = 0;
#pragma omp parallel for schedule(static) reduction(+ : nbad)
    for (int64_t i = 0; i < n; ++i) {
        const char* p = buf + off[i];
        const char* e = buf + off[i + 1];
        double* row = out + i * k;
        uint8_t* fr = found + i * k;
        for (int64_t j = 0; j < k; ++j) {
            row[j] = 0.0;
            fr[j] = 0;
        }
        bool bad = false;
        char tmp[80];
        p = json_ws(p, e);
        if (p >= e || *p != '{') bad = true;
        else ++p;
        p = json_ws(p, e);
        if (!bad && p < e && *p == '}') {
            ++p;
        } else {
            while (!bad) {
                p = json_ws(p, e);
                if (p >= e || *p != '"') { bad = true; break; }
                const char* ks = ++p;
                while (p < e && *p != '"' && *p != '\\') ++p;
                if (p >= e || *p != '"') { bad = true; break; }
                const std::string_view key(ks, (size_t)(p - ks));
                ++p;
                p = json_ws(p, e);
                if (p >= e || *p != ':') { bad = true; break; }
                p = json_ws(p + 1, e);
                auto it = pos.find(key);
                if (p < e && *p == '"') {                   // a string value: only for keys outside the schema
                    if (it != pos.end()) { bad = true; break; }
                    ++p;
                    while (p < e && *p != '"' && *p != '\\') ++p;
                    if (p >= e || *p != '"') { bad = true; break; }
                    ++p;
                } else {
                    const char* vs = p;
                    bool intlike = true;
                    while (p < e && ((*p >= '0' && *p <= '9') || *p == '-' || *p == '+' || *p == '.' || *p == 'e' ||
                                     *p == 'E')) {
                        if (*p == '.' || *p == 'e' || *p == 'E') intlike = false;
                        ++p;
                    }
                    const int64_t len = p - vs;
                    if (len <= 0 || len >= 79) { bad = true; break; }
                    std::memcpy(tmp, vs, (size_t)len);
                    tmp[len] = 0;
                    char* ep = nullptr;
                    double v = strtod(tmp, &ep);
                    if (*ep != 0 || std::isinf(v) || std::isnan(v)) { bad = true; break; }
                    if (intlike && v == 0.0) v = 0.0;           // "-0" is the integer 0
                    if (it != pos.end()) {
                        row[it->second] = v;
                        fr[it->second] = 1;
                    }
                }
                p = json_ws(p, e);
                if (p < e && *p == ',') { ++p; continue; }
                if (p < e && *p == '}') { ++p; break; }
                bad = true;
            }
        }
        if (!bad && json_ws(p, e) != e) bad = true;
        flags[i] = bad ? 1 : 0;
        nbad += bad ? 1 : 0;
    }
    return nbad;
}

// Rows of k doubles with per-column decoration: row i = ropen + [pre_0 v_0 post_0] sep [pre_1 v_1 post_1] ... + rclose,
// v = Double.toString (COLUMNS -> KV "k:v,..." / JSON {"k":"v",...} writers).  out capacity: the caller's bound;
// row_end[i] = end offset of row i.  OpenMP row blocks formatted into per-block slices, then compacted.
extern "C" int64_t alink_java_double_rows_fmt(const double* x, int64_t n, int64_t k, const char* pre,
                                              const int64_t* pre_off, const char* post, const int64_t* post_off,
                                              char sep, const char* ropen, int64_t lo, const char* rclose, int64_t lc,
                                              char* out, int64_t* row_end) {
    int64_t deco = lo + lc + (k > 0 ? k - 1 : 0) + pre_off[k] + post_off[k];
    const int64_t per_row = deco + 26 * k;
    const int64_t rows_per = std::max<int64_t>(1, 8192 / std::max<int64_t>(k, 1));
    const int64_t nb = (n + rows_per - 1) / rows_per;
    std::vector<int64_t> blen(nb);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t r0 = b * rows_per, r1 = std::min(n, r0 + rows_per);
        char* base = out + r0 * per_row;
        int64_t p = 0;
        for (int64_t i = r0; i < r1; ++i) {
            std::memcpy(base + p, ropen, (size_t)lo);
            p += lo;
            for (int64_t j = 0; j < k; ++j) {
                if (j) base[p++] = sep;
                const int64_t a = pre_off[j + 1] - pre_off[j];
                std::memcpy(base + p, pre + pre_off[j], (size_t)a);
                p += a;
                p += java_double_to(x[i * k + j], base + p);
                const int64_t c = post_off[j + 1] - post_off[j];
                std::memcpy(base + p, post + post_off[j], (size_t)c);
                p += c;
            }
            std::memcpy(base + p, rclose, (size_t)lc);
            p += lc;
            row_end[i] = p;
        }
        blen[b] = p;
    }
    int64_t p = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t r0 = b * rows_per, r1 = std::min(n, r0 + rows_per);
        if (p != r0 * per_row) std::memmove(out + p, out + r0 * per_row, (size_t)blen[b]);
        for (int64_t i = r0; i < r1; ++i) row_end[i] += p;
        p += blen[b];
    }
    return p;
}

// CSV / text lines from k packed string columns: row r = col0[r] + delim + col1[r] + ... + col{k-1}[r] + rowdelim,
// written at out + row_off[r] (row_off from the caller's length prefix sum, so rows are independent: OpenMP over
// row blocks).  data[j] / off[j] are column j's bytes and its int64 [n+1] offsets.
extern "C" void alink_join_packed_columns(int64_t k, const uint8_t* const* data, const int64_t* const* off, int64_t n,
                                          const char* delim, int64_t dlen, const char* rowdelim, int64_t rlen,
                                          const int64_t* row_off, uint8_t* out) {
#pragma omp parallel for schedule(static) if (n > 4096)
    for (int64_t r = 0; r < n; ++r) {
        uint8_t* p = out + row_off[r];
        for (int64_t j = 0; j < k; ++j) {
            if (j) { std::memcpy(p, delim, (size_t)dlen); p += dlen; }
            const int64_t a = off[j][r], b = off[j][r + 1];
            std::memcpy(p, data[j] + a, (size_t)(b - a));
            p += b - a;
        }
        std::memcpy(p, rowdelim, (size_t)rlen);
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Top-level member values of JSON objects (JsonValueBatchOp with plain "$.key" paths).  Per document i and key j:
//   kind 0 missing, 1 string without escapes / control bytes (span = its contents), 3 canonical integer literal
//   (span = its text), 4 other number (num = strtod value), 5 true / false (span = its text), 2 anything else
//   (object, array, null, escaped string, "-0": the caller's JSON reader formats it).
// row_ok[i] = 0 when the document is not one well-formed JSON object as this scanner reads it (the caller parses
// it with its lenient reader).  Duplicate members: the last one wins, as a dict-building parser.
namespace {
struct JsonScan {
    const uint8_t* s;
    int64_t n, p;
    bool ws() {
        while (p < n && (s[p] == ' ' || s[p] == '\t' || s[p] == '\n' || s[p] == '\r')) ++p;
        return p < n;
    }
    // string at s[p] == '"': end = index of the closing quote; esc = backslash or control byte inside
    bool str(int64_t& a, int64_t& b, bool& esc) {
        a = ++p;
        esc = false;
        while (p < n && s[p] != '"') {
            if (s[p] == '\\') { esc = true; p += 2; continue; }
            if (s[p] < 0x20) esc = true;
            ++p;
        }
        if (p >= n) return false;
        b = p++;
        return true;
    }
    bool skip_nested() {  // s[p] is '{' or '['
        int depth = 0;
        while (p < n) {
            uint8_t c = s[p];
            if (c == '"') { int64_t a, b; bool e; if (!str(a, b, e)) return false; continue; }
            if (c == '{' || c == '[') ++depth;
            else if (c == '}' || c == ']') { if (--depth == 0) { ++p; return true; } }
            ++p;
        }
        return false;
    }
};
}  // namespace

extern "C" void alink_json_top_values(const uint8_t* buf, const int64_t* off, int64_t n, const uint8_t* kbuf,
                                      const int64_t* koff, int64_t k, int64_t* span, uint8_t* kind, double* num,
                                      uint8_t* row_ok) {
#pragma omp parallel for schedule(dynamic, 4096) if (n > 4096)
    for (int64_t i = 0; i < n; ++i) {
        uint8_t* kd = kind + i * k;
        for (int64_t j = 0; j < k; ++j) kd[j] = 0;
        JsonScan t{buf + off[i], off[i + 1] - off[i], 0};
        bool ok = t.ws() && t.s[t.p] == '{';
        if (ok) {
            ++t.p;
            ok = t.ws();
            if (ok && t.s[t.p] == '}') ++t.p;
            else {
                while (ok) {
                    int64_t ka, kb;
                    bool kesc;
                    if (!(t.s[t.p] == '"' && t.str(ka, kb, kesc)) || kesc) { ok = false; break; }
                    if (!t.ws() || t.s[t.p] != ':') { ok = false; break; }
                    ++t.p;
                    if (!t.ws()) { ok = false; break; }
                    int64_t va = t.p, vb;
                    uint8_t vk;
                    double v = 0;
                    uint8_t c = t.s[t.p];
                    if (c == '"') {
                        int64_t a, b;
                        bool e;
                        if (!t.str(a, b, e)) { ok = false; break; }
                        va = a, vb = b, vk = e ? 2 : 1;
                    } else if (c == '{' || c == '[') {
                        if (!t.skip_nested()) { ok = false; break; }
                        vb = t.p, vk = 2;
                    } else if (c == 't' || c == 'f' || c == 'n') {
                        const char* lit = c == 't' ? "true" : (c == 'f' ? "false" : "null");
                        int64_t L = (int64_t)std::strlen(lit);
                        if (t.p + L > t.n || std::memcmp(t.s + t.p, lit, (size_t)L) != 0) { ok = false; break; }
                        t.p += L;
                        vb = t.p, vk = c == 'n' ? 2 : 5;
                    } else if (c == '-' || (c >= '0' && c <= '9')) {
                        int64_t q = t.p + (c == '-');
                        int64_t d0 = q;
                        while (q < t.n && t.s[q] >= '0' && t.s[q] <= '9') ++q;
                        int64_t nd = q - d0;
                        if (nd == 0 || (nd > 1 && t.s[d0] == '0')) { ok = false; break; }
                        bool isint = true;
                        if (q < t.n && t.s[q] == '.') {
                            isint = false;
                            int64_t f0 = ++q;
                            while (q < t.n && t.s[q] >= '0' && t.s[q] <= '9') ++q;
                            if (q == f0) { ok = false; break; }
                        }
                        if (q < t.n && (t.s[q] == 'e' || t.s[q] == 'E')) {
                            isint = false;
                            ++q;
                            if (q < t.n && (t.s[q] == '+' || t.s[q] == '-')) ++q;
                            int64_t e0 = q;
                            while (q < t.n && t.s[q] >= '0' && t.s[q] <= '9') ++q;
                            if (q == e0) { ok = false; break; }
                        }
                        vb = q;
                        t.p = q;
                        if (isint) {
                            vk = (c == '-' && nd == 1 && t.s[d0] == '0') ? 2 : 3;
                        } else {
                            std::string tmp((const char*)t.s + va, (size_t)(vb - va));
                            v = std::strtod(tmp.c_str(), nullptr);
                            vk = 4;
                        }
                    } else { ok = false; break; }
                    for (int64_t j = 0; j < k; ++j) {
                        int64_t L = koff[j + 1] - koff[j];
                        if (L == kb - ka && std::memcmp(t.s + ka, kbuf + koff[j], (size_t)L) == 0) {
                            kd[j] = vk;
                            span[2 * (i * k + j)] = off[i] + va;
                            span[2 * (i * k + j) + 1] = off[i] + vb;
                            num[i * k + j] = v;
                        }
                    }
                    if (!t.ws()) { ok = false; break; }
                    if (t.s[t.p] == ',') {
                        ++t.p;
                        if (!t.ws()) { ok = false; break; }
                        continue;
                    }
                    if (t.s[t.p] == '}') { ++t.p; break; }
                    ok = false;
                }
            }
            if (ok && t.ws()) ok = false;  // trailing bytes after the object
        }
        row_ok[i] = ok ? 1 : 0;
    }
}
