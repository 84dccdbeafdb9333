// cx_wire.cpp -- JSON wire bridge over the engine.
//
// Answers the reference's GET_SUCC request object (GetSuccHandler,
// abstract_chord_peer.cpp:332-337; handler map chord_peer.cpp:15-40; dispatch
// and error mapping server.h:140-165,194-210) plus a batched form, for a ring
// of peers named "ip:port".  Keys are parsed and every peer's ID / MIN_KEY
// strings are formatted by the engine's GPU hex codec; lookups are cx_route
// calls.  Host code only: a small JSON reader/writer for these objects.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/chordx.h"

namespace {

// ---------------------------------------------------------------- JSON values
struct JVal {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double num = 0;
    std::string str;
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;

    const JVal *get(const char *key) const {
        if (kind != OBJ) return nullptr;
        for (const auto &kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
};

class Reader {
public:
    Reader(const char *p, size_t n) : p_(p), e_(p + n) {}

    bool parse(JVal &out, std::string &err) {
        ws();
        if (!value(out, 0)) {
            err = err_.empty() ? "malformed JSON" : err_;
            return false;
        }
        ws();
        if (p_ != e_) {
            err = "trailing characters after JSON value";
            return false;
        }
        return true;
    }

private:
    const char *p_, *e_;
    std::string err_;

    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
    }
    bool lit(const char *s) {
        const size_t n = std::strlen(s);
        if ((size_t)(e_ - p_) < n || std::memcmp(p_, s, n) != 0) return false;
        p_ += n;
        return true;
    }
    bool value(JVal &v, int depth) {
        if (depth > 64) {
            err_ = "JSON nested too deeply";
            return false;
        }
        if (p_ >= e_) return false;
        switch (*p_) {
        case '{': return object(v, depth);
        case '[': return array(v, depth);
        case '"': v.kind = JVal::STR; return string(v.str);
        case 't': v.kind = JVal::BOOL; v.b = true; return lit("true");
        case 'f': v.kind = JVal::BOOL; v.b = false; return lit("false");
        case 'n': v.kind = JVal::NUL; return lit("null");
        default: return number(v);
        }
    }
    bool number(JVal &v) {
        const char *s = p_;
        if (p_ < e_ && (*p_ == '-' || *p_ == '+')) ++p_;
        while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' ||
                           *p_ == 'E' || *p_ == '-' || *p_ == '+'))
            ++p_;
        if (p_ == s) return false;
        v.kind = JVal::NUM;
        v.num = std::strtod(std::string(s, p_).c_str(), nullptr);
        return true;
    }
    static void utf8(std::string &out, unsigned cp) {
        if (cp < 0x80) {
            out += (char)cp;
        } else if (cp < 0x800) {
            out += (char)(0xC0 | (cp >> 6));
            out += (char)(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12));
            out += (char)(0x80 | ((cp >> 6) & 0x3F));
            out += (char)(0x80 | (cp & 0x3F));
        } else {
            out += (char)(0xF0 | (cp >> 18));
            out += (char)(0x80 | ((cp >> 12) & 0x3F));
            out += (char)(0x80 | ((cp >> 6) & 0x3F));
            out += (char)(0x80 | (cp & 0x3F));
        }
    }
    bool hex4(unsigned &cp) {
        if (e_ - p_ < 4) return false;
        cp = 0;
        for (int i = 0; i < 4; ++i) {
            const char c = *p_++;
            cp <<= 4;
            if (c >= '0' && c <= '9') cp |= (unsigned)(c - '0');
            else if (c >= 'a' && c <= 'f') cp |= (unsigned)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') cp |= (unsigned)(c - 'A' + 10);
            else return false;
        }
        return true;
    }
    bool string(std::string &out) {
        ++p_;  // opening quote
        out.clear();
        while (p_ < e_ && *p_ != '"') {
            if (*p_ != '\\') {
                out += *p_++;
                continue;
            }
            if (++p_ >= e_) return false;
            const char c = *p_++;
            switch (c) {
            case '"': out += '"'; break;
            case '\\': out += '\\'; break;
            case '/': out += '/'; break;
            case 'b': out += '\b'; break;
            case 'f': out += '\f'; break;
            case 'n': out += '\n'; break;
            case 'r': out += '\r'; break;
            case 't': out += '\t'; break;
            case 'u': {
                unsigned cp;
                if (!hex4(cp)) return false;
                if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                    p_ += 2;
                    unsigned lo;
                    if (!hex4(lo)) return false;
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                }
                utf8(out, cp);
                break;
            }
            default: return false;
            }
        }
        if (p_ >= e_) return false;
        ++p_;
        return true;
    }
    bool array(JVal &v, int depth) {
        ++p_;
        v.kind = JVal::ARR;
        ws();
        if (p_ < e_ && *p_ == ']') {
            ++p_;
            return true;
        }
        for (;;) {
            v.arr.emplace_back();
            ws();
            if (!value(v.arr.back(), depth + 1)) return false;
            ws();
            if (p_ < e_ && *p_ == ',') {
                ++p_;
                continue;
            }
            if (p_ < e_ && *p_ == ']') {
                ++p_;
                return true;
            }
            return false;
        }
    }
    bool object(JVal &v, int depth) {
        ++p_;
        v.kind = JVal::OBJ;
        ws();
        if (p_ < e_ && *p_ == '}') {
            ++p_;
            return true;
        }
        for (;;) {
            ws();
            if (p_ >= e_ || *p_ != '"') return false;
            std::string k;
            if (!string(k)) return false;
            ws();
            if (p_ >= e_ || *p_ != ':') return false;
            ++p_;
            ws();
            v.obj.emplace_back(std::move(k), JVal());
            if (!value(v.obj.back().second, depth + 1)) return false;
            ws();
            if (p_ < e_ && *p_ == ',') {
                ++p_;
                continue;
            }
            if (p_ < e_ && *p_ == '}') {
                ++p_;
                return true;
            }
            return false;
        }
    }
};

void put_str(std::string &out, const std::string &s) {
    out += '"';
    for (const unsigned char c : s) {
        switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        default:
            if (c < 0x20) {
                char b[8];
                std::snprintf(b, sizeof(b), "\\u%04x", c);
                out += b;
            } else {
                out += (char)c;
            }
        }
    }
    out += '"';
}

std::string failure(const std::string &msg) {
    std::string r = "{\"ERRORS\":";
    put_str(r, msg);
    r += ",\"SUCCESS\":false}";
    return r;
}

extern "C" int cxi_set_error(int code, const char *msg);  // cx_api.hip

std::string last_error() {
    const char *e = cx_last_error();
    return e ? e : "chordx error";
}

}  // namespace

struct cx_wire {
    cx_ring *ring = nullptr;
    int device = 0;
    std::vector<std::string> ip;       // by ring index
    std::vector<int> port;
    std::vector<std::string> id_hex;   // std::string(id) of each peer
    std::vector<std::string> min_hex;  // std::string(pred.id + 1)
    std::vector<cx_u128> ids;          // ring IDs, ascending
    std::unordered_map<std::string, uint32_t> index;  // "ip:port" -> ring index
};

namespace {

// Parses hex key strings on the GPU; ok[i] = 0 for an invalid string, 2 for
// a raw value >= 2^128.
int parse_keys(const cx_wire *w, const std::vector<const std::string *> &keys,
               std::vector<cx_u128> &out, std::vector<uint8_t> &ok) {
    std::vector<uint64_t> offs(keys.size() + 1, 0);
    std::string bytes;
    for (size_t i = 0; i < keys.size(); ++i) {
        bytes += *keys[i];
        offs[i + 1] = bytes.size();
    }
    out.assign(keys.size(), cx_u128{0, 0});
    ok.assign(keys.size(), 0);
    if (keys.empty()) return CX_OK;
    return cx_hex_parse(reinterpret_cast<const uint8_t *>(bytes.data()), offs.data(), keys.size(),
                        out.data(), ok.data(), CX_MEM_HOST, w->device);
}

inline bool u128_eq(cx_u128 a, cx_u128 b) { return a.lo == b.lo && a.hi == b.hi; }
inline cx_u128 u128_inc(cx_u128 a) { return {a.lo + 1, a.hi + (a.lo == UINT64_MAX ? 1u : 0u)}; }

const char *status_error(uint8_t st) {
    // finger_table.h:129 / chord_peer.cpp:206
    return st == CX_Q_NOT_FOUND ? "ChordKey not found" : "Lookup failed";
}

// Keys whose raw uint256 value is >= 2^128 (ok == 2).  The engine routes
// m = value mod 2^128, which is what every ranged InBetween reads (key.h:
// 116-118); only the point tests (lb == ub, key.h:108-113) see the raw value,
// and it never equals a bound < 2^128.  On the converged ring two point tests
// exist: StoredLocally at a peer whose min_key == id (its predecessor's ID is
// id - 1), and finger 0's range [id+1, id+1] (finger_table.h:177-188).  So
// with x = pred(owner) and m == x.id + 1 (n >= 2):
//   * m == owner.id  -> x and the owner both fail: "ChordKey not found";
//   * otherwise the walk fails at x iff it visits x.  The walk to m and the
//     walk to m - 1 = x.id take the same fingers until a step whose distance
//     m - cur is a power of two (that step jumps straight to the owner), so
//     the walk to m visits x iff hops(m) == hops(x.id) + 1.  The second walk
//     runs on the GPU for just these keys.
// Every other wide key routes as m.  (oracle or_route_raw_batch is the
// literal raw-value walk the wire tests compare against.)
int wide_keys(const cx_wire *w, const std::vector<uint8_t> &ok,
              const std::vector<cx_u128> &kv, const std::vector<uint32_t> &src,
              std::vector<uint32_t> &owner, std::vector<uint8_t> &hops,
              std::vector<uint8_t> &status) {
    const size_t n = w->ids.size();
    if (n < 2) return CX_OK;
    std::vector<size_t> redo;
    for (size_t i = 0; i < kv.size(); ++i) {
        if (ok[i] != 2 || status[i] != CX_Q_OK) continue;
        const uint32_t o = owner[i], x = (uint32_t)((o + n - 1) % n);
        if (!u128_eq(u128_inc(w->ids[x]), kv[i])) continue;
        if (u128_eq(w->ids[o], kv[i])) {
            status[i] = CX_Q_NOT_FOUND;
            owner[i] = CX_NONE;
        } else {
            redo.push_back(i);
        }
    }
    if (redo.empty()) return CX_OK;
    std::vector<cx_u128> k2(redo.size());
    std::vector<uint32_t> s2(redo.size()), o2(redo.size());
    std::vector<uint8_t> h2(redo.size()), st2(redo.size());
    for (size_t j = 0; j < redo.size(); ++j) {
        const size_t i = redo[j];
        k2[j] = w->ids[(owner[i] + n - 1) % n];
        s2[j] = src[i];
    }
    const int e = cx_route(w->ring, s2.data(), k2.data(), redo.size(), o2.data(), h2.data(),
                           st2.data(), CX_MEM_HOST);
    if (e != CX_OK) return e;
    for (size_t j = 0; j < redo.size(); ++j) {
        const size_t i = redo[j];
        if (st2[j] == CX_Q_OK && hops[i] == h2[j] + 1) {
            status[i] = CX_Q_NOT_FOUND;
            owner[i] = CX_NONE;
        }
    }
    return CX_OK;
}

void peer_fields(const cx_wire *w, uint32_t o, std::string &r) {
    r += "\"ID\":\"" + w->id_hex[o] + "\",\"IP_ADDR\":";
    put_str(r, w->ip[o]);
    r += ",\"MIN_KEY\":\"" + w->min_hex[o] + "\",\"PORT\":" + std::to_string(w->port[o]);
}

std::string handle(cx_wire *w, const JVal &req) {
    const JVal *cmd = req.get("COMMAND");
    const std::string c = (cmd && cmd->kind == JVal::STR) ? cmd->str : "";
    const bool batch = c == "GET_SUCC_BATCH";
    if (c != "GET_SUCC" && !batch) return failure("Invalid command.");  // server.h:200-203

    std::vector<const std::string *> keys;
    if (batch) {
        const JVal *ks = req.get("KEYS");
        if (!ks || ks->kind != JVal::ARR) return failure("GET_SUCC_BATCH needs a KEYS array");
        for (const auto &k : ks->arr) {
            if (k.kind != JVal::STR) return failure("KEYS entries must be hex strings");
            keys.push_back(&k.str);
        }
    } else {
        const JVal *k = req.get("KEY");
        if (!k || k->kind != JVal::STR) return failure("GET_SUCC needs a KEY string");
        keys.push_back(&k->str);
    }
    // source peers: "SRC" (one) or "SRCS" (one per key); default ring index 0
    std::vector<uint32_t> src(keys.size(), 0);
    const JVal *s1 = req.get("SRC"), *sn = batch ? req.get("SRCS") : nullptr;
    auto peer_of = [&](const JVal &v, uint32_t &out) {
        if (v.kind != JVal::STR) return false;
        auto it = w->index.find(v.str);
        if (it == w->index.end()) return false;
        out = it->second;
        return true;
    };
    if (s1) {
        uint32_t p;
        if (!peer_of(*s1, p)) return failure("SRC is not a peer of this ring");
        for (auto &x : src) x = p;
    }
    if (sn) {
        if (sn->kind != JVal::ARR || sn->arr.size() != keys.size())
            return failure("SRCS must list one peer per key");
        for (size_t i = 0; i < keys.size(); ++i)
            if (!peer_of(sn->arr[i], src[i])) return failure("SRCS entry is not a peer of this ring");
    }

    std::vector<cx_u128> kv;
    std::vector<uint8_t> ok;
    if (parse_keys(w, keys, kv, ok) != CX_OK) return failure(last_error());
    const size_t q = keys.size();
    std::vector<uint32_t> owner(q, CX_NONE);
    std::vector<uint8_t> hops(q, 0), status(q, 0);
    if (q && cx_route(w->ring, src.data(), kv.data(), q, owner.data(), hops.data(),
                      status.data(), CX_MEM_HOST) != CX_OK)
        return failure(last_error());
    if (wide_keys(w, ok, kv, src, owner, hops, status) != CX_OK) return failure(last_error());

    if (!batch) {
        if (!ok[0]) return failure("invalid hex key: \"" + *keys[0] + "\"");
        if (status[0] != CX_Q_OK) return failure(status_error(status[0]));
        std::string r = "{";
        peer_fields(w, owner[0], r);
        r += ",\"SUCCESS\":true}";
        return r;
    }
    std::string r = "{\"RESULTS\":[";
    r.reserve(q * 150 + 32);
    for (size_t i = 0; i < q; ++i) {
        if (i) r += ',';
        if (!ok[i]) {
            r += failure("invalid hex key: \"" + *keys[i] + "\"");
        } else if (status[i] != CX_Q_OK) {
            r += failure(status_error(status[i]));
        } else {
            r += '{';
            r += "\"HOPS\":" + std::to_string(hops[i]) + ',';
            peer_fields(w, owner[i], r);
            r += '}';
        }
    }
    r += "],\"SUCCESS\":true}";
    return r;
}

}  // namespace

extern "C" {

int cx_wire_create(const char *const *addrs, size_t n, int device, cx_wire **out) {
    if (!addrs || !out || n == 0) return cxi_set_error(CX_E_INVALID, "no peer names");
    *out = nullptr;
    cx_wire *w = new cx_wire();
    w->device = device;
    int rc = [&]() -> int {
        std::vector<uint64_t> offs(n + 1, 0);
        std::string bytes;
        std::vector<std::string> names(n);
        for (size_t i = 0; i < n; ++i) {
            if (!addrs[i]) return cxi_set_error(CX_E_INVALID, "null peer name");
            names[i] = addrs[i];
            bytes += names[i];
            offs[i + 1] = bytes.size();
        }
        std::vector<cx_u128> ids(n);
        int e = cx_uuid5_dns(reinterpret_cast<const uint8_t *>(bytes.data()), offs.data(), n,
                             ids.data(), CX_MEM_HOST, device);
        if (e) return e;
        if ((e = cx_ring_create(ids.data(), n, CX_MEM_HOST, device, &w->ring))) return e;
        size_t m = 0;
        cx_ring_size(w->ring, &m);
        if (m != n)  // two names hash to one ID (remote_peer_list.cpp:56-58)
            return cxi_set_error(CX_E_INVALID, "peer names repeat (equal IDs)");
        std::vector<uint32_t> idx(n);
        if ((e = cx_successor(w->ring, ids.data(), n, idx.data(), CX_MEM_HOST))) return e;
        w->ip.assign(n, "");
        w->port.assign(n, 0);
        for (size_t i = 0; i < n; ++i) {
            const std::string &a = names[i];
            const size_t colon = a.rfind(':');
            w->ip[idx[i]] = colon == std::string::npos ? a : a.substr(0, colon);
            w->port[idx[i]] = colon == std::string::npos ? 0 : std::atoi(a.c_str() + colon + 1);
            w->index[a] = idx[i];
        }
        // ID and MIN_KEY = pred.id + 1 of every peer, formatted by the GPU codec
        std::vector<cx_u128> &sorted = w->ids, both(2 * n);
        sorted.assign(n, cx_u128{0, 0});
        if ((e = cx_ring_ids(w->ring, sorted.data(), CX_MEM_HOST))) return e;
        for (size_t i = 0; i < n; ++i) {
            const cx_u128 p = sorted[(i + n - 1) % n];
            cx_u128 mk = {p.lo + 1, p.hi + (p.lo == UINT64_MAX ? 1u : 0u)};
            both[i] = sorted[i];
            both[n + i] = mk;
        }
        std::vector<char> txt(2 * n * 32);
        std::vector<uint8_t> len(2 * n);
        if ((e = cx_hex_format(both.data(), 2 * n, txt.data(), len.data(), CX_MEM_HOST, device)))
            return e;
        w->id_hex.resize(n);
        w->min_hex.resize(n);
        for (size_t i = 0; i < n; ++i) {
            w->id_hex[i].assign(&txt[32 * i], len[i]);
            w->min_hex[i].assign(&txt[32 * (n + i)], len[n + i]);
        }
        return cx_fingers_build(w->ring, nullptr, CX_MEM_HOST);
    }();
    if (rc) {
        if (w->ring) cx_ring_destroy(w->ring);
        delete w;
        return rc;
    }
    *out = w;
    return CX_OK;
}

int cx_wire_destroy(cx_wire *wire) {
    if (!wire) return CX_OK;
    int rc = cx_ring_destroy(wire->ring);
    delete wire;
    return rc;
}

int cx_wire_ring(const cx_wire *wire, const cx_ring **ring) {
    if (!wire || !ring) return cxi_set_error(CX_E_INVALID, "null argument");
    *ring = wire->ring;
    return CX_OK;
}

int cx_wire_handle(cx_wire *wire, const char *request, size_t len, char **response,
                   size_t *response_len) {
    if (!wire || !request || !response) return cxi_set_error(CX_E_INVALID, "null argument");
    JVal req;
    std::string err, r;
    Reader rd(request, len);
    if (!rd.parse(req, err)) r = failure(err);  // server.h:162-165
    else if (req.kind != JVal::OBJ) r = failure("request must be a JSON object");
    else r = handle(wire, req);
    char *buf = static_cast<char *>(std::malloc(r.size() + 1));
    if (!buf) return cxi_set_error(CX_E_NOMEM, "out of host memory");
    std::memcpy(buf, r.data(), r.size());
    buf[r.size()] = 0;
    *response = buf;
    if (response_len) *response_len = r.size();
    return CX_OK;
}

void cx_wire_free(char *response) { std::free(response); }

}  // extern "C"
