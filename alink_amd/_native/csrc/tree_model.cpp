// Tree-model table -> flat forest arrays, in one native pass (no per-node Python objects).
//
// Input: the tree rows of a tree model table (TreeModelDataConverter.serializeModel,
// A/operator/common/tree/TreeModelDataConverter.java): one JSON object per node,
//   {"node":{"featureIndex":f,"gain":g,"counter":{"weightSum":w,"numInst":n,"distributions":[...]},
//            "categoricalSplit":[...],"continuousSplit":t},"id":i,"nextIds":[...]}
// (Gson without nulls: any member may be absent; member order is not relied on).  Trees are given as string
// ranges [tree_lo[t], tree_lo[t+1]); node i of tree t lands at flat index tree_lo[t] + i (ids are the
// serializer's BFS numbering: children of a node are consecutive ids, which the walk kernels rely on).
//
// Outputs per flat node (nstr entries): feat (featureIndex, -1 = leaf / absent), thr (continuousSplit), first
// child flat index (-1 for a leaf), nchild, wsum (counter.weightSum, 0 without a counter), the leaf distribution
// (dist [nstr][nd], zero padded; dist_len = its length, -1 without one) and the categorical map (cat_len = its
// length, -1 without one; values concatenated in node order into catbuf).
//
// alink_tree_flatten returns 0, or 1 + the index of the first string it cannot take (the caller then uses the
// generic JSON path), -1 for inconsistent tree ranges / ids, or -2 when the caller's dist / categorical buffers are
// too small (the sizes it needs are returned; alink_tree_scan computes them up front as well).
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

struct Cursor {
    const char* p;
    const char* e;
    bool bad = false;
};

inline void ws(Cursor& c) {
    while (c.p < c.e && (*c.p == ' ' || *c.p == '\t' || *c.p == '\n' || *c.p == '\r')) ++c.p;
}

inline bool eat(Cursor& c, char ch) {
    ws(c);
    if (c.p < c.e && *c.p == ch) {
        ++c.p;
        return true;
    }
    return false;
}

// a JSON number (or the Gson tokens NaN / Infinity / -Infinity) as a double
double num(Cursor& c) {
    ws(c);
    const char* s = c.p;
    while (c.p < c.e && ((*c.p >= '0' && *c.p <= '9') || *c.p == '-' || *c.p == '+' || *c.p == '.' || *c.p == 'e' ||
                         *c.p == 'E' || *c.p == 'N' || *c.p == 'a' || *c.p == 'I' || *c.p == 'n' || *c.p == 'f' ||
                         *c.p == 'i' || *c.p == 't' || *c.p == 'y'))
        ++c.p;
    const size_t len = (size_t)(c.p - s);
    if (len == 0 || len >= 64) {
        c.bad = true;
        return 0.0;
    }
    char tmp[64];
    std::memcpy(tmp, s, len);
    tmp[len] = 0;
    if (!std::strcmp(tmp, "NaN")) return NAN;
    if (!std::strcmp(tmp, "Infinity")) return INFINITY;
    if (!std::strcmp(tmp, "-Infinity")) return -INFINITY;
    char* ep = nullptr;
    const double v = std::strtod(tmp, &ep);
    if (*ep != 0) c.bad = true;
    return v;
}

// key of the next member ("..." then ':'); false at the closing brace
bool key(Cursor& c, const char*& ks, size_t& kl) {
    ws(c);
    if (c.p < c.e && *c.p == '}') {
        ++c.p;
        return false;
    }
    if (c.p >= c.e || *c.p != '"') {
        c.bad = true;
        return false;
    }
    ks = ++c.p;
    while (c.p < c.e && *c.p != '"') {
        if (*c.p == '\\') ++c.p;
        ++c.p;
    }
    if (c.p >= c.e) {
        c.bad = true;
        return false;
    }
    kl = (size_t)(c.p - ks);
    ++c.p;
    if (!eat(c, ':')) c.bad = true;
    return !c.bad;
}

inline bool is(const char* ks, size_t kl, const char* lit) { return kl == std::strlen(lit) && !std::memcmp(ks, lit, kl); }

void skip_value(Cursor& c);

void skip_string(Cursor& c) {
    ++c.p;
    while (c.p < c.e && *c.p != '"') {
        if (*c.p == '\\') ++c.p;
        ++c.p;
    }
    if (c.p >= c.e) c.bad = true;
    else ++c.p;
}

void skip_value(Cursor& c) {
    ws(c);
    if (c.p >= c.e) {
        c.bad = true;
        return;
    }
    const char ch = *c.p;
    if (ch == '"') return skip_string(c);
    if (ch == '{' || ch == '[') {
        const char close = ch == '{' ? '}' : ']';
        ++c.p;
        ws(c);
        if (c.p < c.e && *c.p == close) {
            ++c.p;
            return;
        }
        while (!c.bad) {
            if (ch == '{') {
                ws(c);
                if (c.p >= c.e || *c.p != '"') { c.bad = true; return; }
                skip_string(c);
                if (!eat(c, ':')) { c.bad = true; return; }
            }
            skip_value(c);
            if (eat(c, ',')) continue;
            if (eat(c, close)) return;
            c.bad = true;
        }
        return;
    }
    if (c.e - c.p >= 4 && (!std::memcmp(c.p, "true", 4) || !std::memcmp(c.p, "null", 4))) {
        c.p += 4;
        return;
    }
    if (c.e - c.p >= 5 && !std::memcmp(c.p, "false", 5)) {
        c.p += 5;
        return;
    }
    num(c);
}

// a JSON array of numbers; calls f(value) per element; returns the count (-1 for null)
template <typename F>
int64_t num_array(Cursor& c, F f) {
    ws(c);
    if (c.e - c.p >= 4 && !std::memcmp(c.p, "null", 4)) {
        c.p += 4;
        return -1;
    }
    if (!eat(c, '[')) {
        c.bad = true;
        return 0;
    }
    int64_t n = 0;
    if (eat(c, ']')) return 0;
    while (!c.bad) {
        f(num(c));
        ++n;
        if (eat(c, ',')) continue;
        if (eat(c, ']')) break;
        c.bad = true;
    }
    return n;
}

struct NodeOut {
    int64_t feat = -1, num_inst = 0, id = -1, first = -1, nchild = 0, dist_len = -1, cat_len = -1;
    double gain = 0.0, thr = 0.0, wsum = 0.0;
    bool contiguous = true;
};

// parse one node string; dist/cat values go through the sinks (nullptr: counted only)
template <typename DS, typename CS>
bool parse_node(const char* s, const char* e, NodeOut& o, DS dist_sink, CS cat_sink) {
    Cursor c{s, e};
    if (!eat(c, '{')) return false;
    const char* ks;
    size_t kl;
    while (key(c, ks, kl)) {
        if (is(ks, kl, "node")) {
            ws(c);
            if (c.e - c.p >= 4 && !std::memcmp(c.p, "null", 4)) {
                c.p += 4;
            } else {
                if (!eat(c, '{')) return false;
                const char* k2;
                size_t l2;
                while (key(c, k2, l2)) {
                    if (is(k2, l2, "featureIndex")) o.feat = (int64_t)num(c);
                    else if (is(k2, l2, "gain")) o.gain = num(c);
                    else if (is(k2, l2, "continuousSplit")) o.thr = num(c);
                    else if (is(k2, l2, "categoricalSplit")) {
                        o.cat_len = num_array(c, [&](double v) { cat_sink((int32_t)v); });
                    } else if (is(k2, l2, "counter")) {
                        ws(c);
                        if (c.e - c.p >= 4 && !std::memcmp(c.p, "null", 4)) {
                            c.p += 4;
                        } else {
                            if (!eat(c, '{')) return false;
                            const char* k3;
                            size_t l3;
                            while (key(c, k3, l3)) {
                                if (is(k3, l3, "weightSum")) o.wsum = num(c);
                                else if (is(k3, l3, "numInst")) o.num_inst = (int64_t)num(c);
                                else if (is(k3, l3, "distributions")) {
                                    int64_t j = 0;
                                    o.dist_len = num_array(c, [&](double v) { dist_sink(j++, v); });
                                } else skip_value(c);
                                if (c.bad) return false;
                                if (!eat(c, ',')) {
                                    if (!eat(c, '}')) return false;
                                    break;
                                }
                            }
                        }
                    } else skip_value(c);
                    if (c.bad) return false;
                    if (!eat(c, ',')) {
                        if (!eat(c, '}')) return false;
                        break;
                    }
                }
            }
        } else if (is(ks, kl, "id")) {
            o.id = (int64_t)num(c);
        } else if (is(ks, kl, "nextIds")) {
            int64_t prev = -2;
            o.nchild = num_array(c, [&](double v) {
                const int64_t id = (int64_t)v;
                if (prev == -2) o.first = id;
                else if (id != prev + 1) o.contiguous = false;
                prev = id;
            });
            if (o.nchild < 0) o.nchild = 0;
        } else {
            skip_value(c);
        }
        if (c.bad) return false;
        if (!eat(c, ',')) {
            if (!eat(c, '}')) return false;
            break;
        }
    }
    ws(c);
    return !c.bad && c.p == c.e;
}

}  // namespace

extern "C" {

// sizes: *max_dist = longest distributions array (0 if none), *cat_total = categorical values over all nodes
int64_t alink_tree_scan(const char* buf, const int64_t* off, int64_t nstr, int64_t* max_dist, int64_t* cat_total) {
    int64_t bad = nstr + 1, md = 0, ct = 0;
#pragma omp parallel for schedule(static) reduction(min : bad) reduction(max : md) reduction(+ : ct)
    for (int64_t i = 0; i < nstr; ++i) {
        NodeOut o;
        if (!parse_node(buf + off[i], buf + off[i + 1], o, [](int64_t, double) {}, [](int32_t) {}) ||
            !o.contiguous || o.id < 0) {
            if (i < bad) bad = i;
            continue;
        }
        if (o.dist_len > md) md = o.dist_len;
        if (o.cat_len > 0) ct += o.cat_len;
    }
    *max_dist = md;
    *cat_total = ct;
    return bad <= nstr - 1 ? bad + 1 : 0;
}

// flat arrays (see the header); nd = distribution width of dist, cat_off [nstr] receives each node's offset into
// catbuf.  Node i of tree t must carry id = i - tree_lo[t] (the serializer's order).  When nd or cat_cap is too
// small nothing is written past the first pass: the call returns -2 with *need_nd / *need_cat set (call again).
int64_t alink_tree_flatten(const char* buf, const int64_t* off, int64_t nstr, const int64_t* tree_lo, int64_t ntrees,
                           int64_t nd, int32_t* feat, double* thr, int32_t* first, int32_t* nchild, double* wsum,
                           double* dist, int32_t* dist_len, int32_t* cat_len, int64_t* cat_off, int32_t* catbuf,
                           int64_t cat_cap, int64_t* need_nd, int64_t* need_cat) {
    if (tree_lo[0] != 0 || tree_lo[ntrees] != nstr) return -1;
    std::vector<int64_t> tree_of((size_t)nstr);
    for (int64_t t = 0; t < ntrees; ++t) {
        if (tree_lo[t + 1] < tree_lo[t]) return -1;
        for (int64_t i = tree_lo[t]; i < tree_lo[t + 1]; ++i) tree_of[(size_t)i] = t;
    }
    // categorical counts and the widest distribution first (exact offsets), then the full parse in parallel
    std::vector<int64_t> clen((size_t)nstr + 1, 0);
    int64_t bad = nstr + 1, md = 0;
#pragma omp parallel for schedule(static) reduction(min : bad) reduction(max : md)
    for (int64_t i = 0; i < nstr; ++i) {
        NodeOut o;
        if (!parse_node(buf + off[i], buf + off[i + 1], o, [](int64_t, double) {}, [](int32_t) {})) {
            if (i < bad) bad = i;
            continue;
        }
        clen[(size_t)i + 1] = o.cat_len > 0 ? o.cat_len : 0;
        if (o.dist_len > md) md = o.dist_len;
    }
    if (bad <= nstr - 1) return bad + 1;
    for (int64_t i = 0; i < nstr; ++i) clen[(size_t)i + 1] += clen[(size_t)i];
    *need_nd = md;
    *need_cat = clen[(size_t)nstr];
    if (clen[(size_t)nstr] > cat_cap || md > nd) return -2;
    int64_t bad_id = 0;
#pragma omp parallel for schedule(static) reduction(min : bad) reduction(+ : bad_id)
    for (int64_t i = 0; i < nstr; ++i) {
        NodeOut o;
        double* drow = dist + i * nd;
        for (int64_t j = 0; j < nd; ++j) drow[j] = 0.0;
        int64_t cpos = clen[(size_t)i];
        const bool ok = parse_node(
            buf + off[i], buf + off[i + 1], o, [&](int64_t j, double v) { if (j < nd) drow[j] = v; },
            [&](int32_t v) { catbuf[cpos++] = v; });
        if (!ok) {
            if (i < bad) bad = i;
            continue;
        }
        const int64_t t = tree_of[(size_t)i], base = tree_lo[t], size = tree_lo[t + 1] - base;
        // ids must be the node's position in its tree (BFS numbering) and children inside the tree
        if (o.id != i - base || !o.contiguous || (o.nchild > 0 && (o.first <= o.id || o.first + o.nchild > size)) ||
            o.dist_len > nd) {
            bad_id += 1;
            continue;
        }
        const bool leaf = o.feat == -1;
        feat[i] = (int32_t)o.feat;
        thr[i] = o.thr;
        first[i] = leaf || o.nchild == 0 ? -1 : (int32_t)(base + o.first);
        nchild[i] = leaf ? 0 : (int32_t)o.nchild;
        wsum[i] = o.wsum;
        dist_len[i] = (int32_t)o.dist_len;
        cat_len[i] = (int32_t)o.cat_len;
        cat_off[i] = clen[(size_t)i];
    }
    if (bad <= nstr - 1) return bad + 1;
    return bad_id ? -1 : 0;
}

}  // extern "C"
