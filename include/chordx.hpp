// chordx.hpp -- C++ face of the chordx C ABI, mirroring the reference's
// lookup-path classes (header-only; link with libchordx.so).
//
//   reference (Patrick-McKeever/P2P-DHTs)            chordx.hpp
//   ----------------------------------------------   ----------------------------------
//   ChordKey (key.h:355), hex ctor (key.h:73-75)     chordx::Key, Key::FromHex
//   ChordKey::InBetween (key.h:103-131)              Key::InBetween (GPU, raw uint256)
//   std::string(ChordKey) (key.h:41-47,199-201)      Key::Str (hex, no leading zeros)
//   converged ring of ChordPeers                     chordx::Ring (sorted, de-duplicated IDs)
//   AbstractChordPeer::PopulateFingerTable           Ring::PopulateFingerTable
//     (abstract_chord_peer.cpp:564-613)
//   FingerTable::GetNthEntry / EditNthFinger         Ring::FingerTable / Ring::EditFingers
//     (finger_table.h:102-141)
//   AbstractChordPeer::GetSuccessor(key)             Ring::GetSuccessor(src, key) -> {owner, hops}
//     (abstract_chord_peer.cpp:318-330)
//   AbstractChordPeer::GetPredecessor(key)           Ring::GetPredecessor(key)
//     (abstract_chord_peer.cpp:380-421)
//   AbstractChordPeer::GetNSuccessors(key, n)        Ring::GetNSuccessors(key, n)
//     (abstract_chord_peer.cpp:345-373)
//   DHashPeer::Create's replica check                Ring::CheckReplicas(n, m)
//     (dhash_peer.cpp:109-112)
//
// Errors are thrown as chordx::Error (a std::runtime_error carrying the cx_err
// code), with the reference's messages where it has one.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "chordx.h"

namespace chordx {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string &msg) : std::runtime_error(msg), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void check(int rc) {
    if (rc != CX_OK) throw Error(rc, cx_last_error());
}

// A 128-bit ring value (canonical ChordKey).
struct Key {
    uint64_t lo = 0, hi = 0;

    Key() = default;
    Key(uint64_t hi_, uint64_t lo_) : lo(lo_), hi(hi_) {}
    explicit Key(unsigned __int128 v) : lo((uint64_t)v), hi((uint64_t)(v >> 64)) {}

    // ChordKey(hex, hashed = true): uint256_t("0x" + key) (key.h:73-75), mod 2^128.
    static Key FromHex(const std::string &s) {
        unsigned __int128 v = 0;
        for (char c : s) {
            int d;
            if (c >= '0' && c <= '9') d = c - '0';
            else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
            else throw Error(CX_E_INVALID, "invalid hex key: " + s);
            v = (v << 4) | (unsigned)d;
        }
        return Key(v);
    }

    unsigned __int128 value() const { return ((unsigned __int128)hi << 64) | lo; }

    // IntToHexStr (key.h:41-47): lowercase, no leading zeros.
    std::string Str() const {
        static const char *hx = "0123456789abcdef";
        unsigned __int128 v = value();
        if (v == 0) return "0";
        std::string r;
        while (v) {
            r.insert(r.begin(), hx[(unsigned)(v & 15)]);
            v >>= 4;
        }
        return r;
    }

    // ChordKey::InBetween(lb, ub, inclusive), evaluated by the engine.
    bool InBetween(const Key &lb, const Key &ub, bool inclusive = true) const {
        cx_u256 v{{lo, hi, 0, 0}}, l{{lb.lo, lb.hi, 0, 0}}, u{{ub.lo, ub.hi, 0, 0}};
        uint8_t out = 0;
        check(cx_in_between(&v, &l, &u, 1, inclusive ? 1 : 0, &out, CX_MEM_HOST));
        return out != 0;
    }

    friend bool operator==(const Key &a, const Key &b) { return a.lo == b.lo && a.hi == b.hi; }
    friend bool operator!=(const Key &a, const Key &b) { return !(a == b); }
    friend bool operator<(const Key &a, const Key &b) { return a.value() < b.value(); }

    cx_u128 cx() const { return cx_u128{lo, hi}; }
};

struct Lookup {
    uint32_t owner;  // ring index of the peer whose StoredLocally(key) holds
    uint8_t hops;    // GET_SUCC requests sent (0 if the source stores the key)
    uint8_t status;  // cx_qstatus: CX_Q_OK, _HOPCAP, _BADPEER, _FAILED, _NOT_FOUND
};

// A converged ring of peers on one GPU.
class Ring {
public:
    explicit Ring(const std::vector<Key> &ids, int device = 0) {
        std::vector<cx_u128> v;
        v.reserve(ids.size());
        for (const Key &k : ids) v.push_back(k.cx());
        check(cx_ring_create(v.data(), v.size(), CX_MEM_HOST, device, &h_));
    }
    explicit Ring(cx_ring *adopt) : h_(adopt) {}
    Ring(const Ring &) = delete;
    Ring &operator=(const Ring &) = delete;
    Ring(Ring &&o) noexcept : h_(o.h_) { o.h_ = nullptr; }
    ~Ring() {
        if (h_) cx_ring_destroy(h_);
    }

    cx_ring *handle() const { return h_; }

    size_t Size() const {
        size_t n = 0;
        check(cx_ring_size(h_, &n));
        return n;
    }

    std::vector<Key> Ids() const {
        std::vector<cx_u128> v(Size());
        check(cx_ring_ids(h_, v.data(), CX_MEM_HOST));
        std::vector<Key> r;
        r.reserve(v.size());
        for (const cx_u128 &k : v) r.emplace_back(k.hi, k.lo);
        return r;
    }

    // Index of a peer ID in the ring (throws "ChordKey not found" if absent).
    uint32_t IndexOf(const Key &id) const {
        const uint32_t s = Owner(id);
        if (Ids()[s] != id) throw Error(CX_E_NOT_FOUND, "ChordKey not found");
        return s;
    }

    // Owner (converged StoredLocally) of each key.
    std::vector<uint32_t> Successors(const std::vector<Key> &keys) const {
        std::vector<cx_u128> k = pack(keys);
        std::vector<uint32_t> out(keys.size());
        check(cx_successor(h_, k.data(), k.size(), out.data(), CX_MEM_HOST));
        return out;
    }
    uint32_t Owner(const Key &key) const { return Successors({key})[0]; }

    // GetPredecessor on the converged ring (abstract_chord_peer.cpp:380-421):
    // the predecessor of each key's owner (a lone peer answers itself).
    std::vector<uint32_t> GetPredecessors(const std::vector<Key> &keys) const {
        std::vector<cx_u128> k = pack(keys);
        std::vector<uint32_t> out(keys.size());
        check(cx_predecessor(h_, k.data(), k.size(), out.data(), CX_MEM_HOST));
        return out;
    }
    uint32_t GetPredecessor(const Key &key) const { return GetPredecessors({key})[0]; }

    void PopulateFingerTable() { check(cx_fingers_build(h_, nullptr, CX_MEM_HOST)); }

    // Row-major n x 128 finger successors (peer indices).
    std::vector<uint32_t> FingerTable() {
        std::vector<uint32_t> F(Size() * CX_FINGERS);
        check(cx_fingers_build(h_, F.data(), CX_MEM_HOST));
        return F;
    }

    // Replace the whole table (EditNthFinger / AdjustFingers / ReplaceDeadPeer
    // results); routes then follow ForwardRequest literally.
    void EditFingers(const std::vector<uint32_t> &F) {
        if (F.size() != Size() * CX_FINGERS) throw Error(CX_E_INVALID, "finger table size");
        check(cx_fingers_upload(h_, F.data(), CX_MEM_HOST));
    }

    // Liveness and successors_ lists (n x ns, CX_NONE-padded; nullptr = the
    // converged lists) for ForwardRequest's dead-finger branch; rule =
    // CX_FWD_CHORD (chord_peer.cpp:201-208) or CX_FWD_DHASH (dhash_peer.cpp:516-526).
    // Both nullptr: reset to "all alive, converged lists" (the converged walk).
    void SetLiveness(const std::vector<uint8_t> *alive, const std::vector<uint32_t> *succs, int ns,
                     int rule = CX_FWD_CHORD) {
        if (alive && alive->size() != Size()) throw Error(CX_E_INVALID, "alive size");
        if (succs && succs->size() != Size() * (size_t)ns) throw Error(CX_E_INVALID, "succs size");
        check(cx_liveness_upload(h_, alive ? alive->data() : nullptr,
                                 succs ? succs->data() : nullptr, ns, rule, CX_MEM_HOST));
    }

    // min_key_ / predecessor_ per peer (CX_NONE = predecessor not set).
    void SetPeerState(const std::vector<Key> *min_keys, const std::vector<uint32_t> *preds) {
        std::vector<cx_u128> mk;
        if (min_keys) mk = pack(*min_keys);
        check(cx_peer_state_upload(h_, min_keys ? mk.data() : nullptr,
                                   preds ? preds->data() : nullptr, CX_MEM_HOST));
    }

    // Batched GetSuccessor issued at peers src[i].
    std::vector<Lookup> Route(const std::vector<uint32_t> &src, const std::vector<Key> &keys) const {
        if (src.size() != keys.size()) throw Error(CX_E_INVALID, "src/keys size mismatch");
        std::vector<cx_u128> k = pack(keys);
        std::vector<uint32_t> owner(keys.size());
        std::vector<uint8_t> hops(keys.size()), st(keys.size());
        check(cx_route(h_, src.data(), k.data(), k.size(), owner.data(), hops.data(), st.data(),
                       CX_MEM_HOST));
        std::vector<Lookup> r(keys.size());
        for (size_t i = 0; i < r.size(); ++i) r[i] = Lookup{owner[i], hops[i], st[i]};
        return r;
    }

    // GetSuccessor(key) at peer src, throwing the reference's messages:
    // "Lookup failed" (chord_peer.cpp:206, dhash_peer.cpp:524; also the walk
    // livelocking past the hop cap), "ChordKey not found" (finger_table.h:129).
    Lookup GetSuccessor(uint32_t src, const Key &key) const {
        Lookup l = Route({src}, {key})[0];
        if (l.status == CX_Q_HOPCAP || l.status == CX_Q_FAILED)
            throw Error(CX_E_LOOKUP_FAILED, "Lookup failed");
        if (l.status == CX_Q_NOT_FOUND) throw Error(CX_E_NOT_FOUND, "ChordKey not found");
        if (l.status == CX_Q_BADPEER) throw Error(CX_E_INVALID, "Peer is down.");
        return l;
    }

    std::vector<uint32_t> GetNSuccessors(const Key &key, int n) const {
        std::vector<uint32_t> lists(n);
        uint8_t count = 0;
        cx_u128 k = key.cx();
        check(cx_nsucc(h_, &k, 1, n, lists.data(), &count, CX_MEM_HOST));
        lists.resize(count);
        return lists;
    }

    // DHashPeer::Create's precondition (n successors, m needed to decode).
    void CheckReplicas(int n = 14, int m = 10) const { check(cx_dhash_check(h_, n, m)); }

    // Batched join/leave: the new ring and old_to_new (CX_NONE = left).
    std::pair<Ring, std::vector<uint32_t>> Churn(const std::vector<Key> &joins,
                                                 const std::vector<Key> &leaves) const {
        std::vector<cx_u128> j = pack(joins), l = pack(leaves);
        std::vector<uint32_t> o2n(Size());
        cx_ring *nr = nullptr;
        check(cx_churn(h_, j.data(), j.size(), l.data(), l.size(), CX_MEM_HOST, &nr, o2n.data()));
        return {Ring(nr), std::move(o2n)};
    }

private:
    static std::vector<cx_u128> pack(const std::vector<Key> &keys) {
        std::vector<cx_u128> v;
        v.reserve(keys.size());
        for (const Key &k : keys) v.push_back(k.cx());
        return v;
    }
    cx_ring *h_ = nullptr;
};

// Wire bridge (cx_wire_*): answers GET_SUCC request objects for a ring of
// peers named "ip:port" (chord_peer.cpp:15-40, server.h:194-210).
class Wire {
public:
    Wire(const std::vector<std::string> &addrs, int device = 0) {
        std::vector<const char *> p;
        for (const auto &a : addrs) p.push_back(a.c_str());
        check(cx_wire_create(p.data(), p.size(), device, &h_));
    }
    ~Wire() { cx_wire_destroy(h_); }
    Wire(const Wire &) = delete;
    Wire &operator=(const Wire &) = delete;

    // JSON request text -> JSON response text.
    std::string Handle(const std::string &request) {
        char *out = nullptr;
        size_t len = 0;
        check(cx_wire_handle(h_, request.data(), request.size(), &out, &len));
        std::string r(out, len);
        cx_wire_free(out);
        return r;
    }

private:
    cx_wire *h_ = nullptr;
};

// Rabin IDA (cx_ida_*): DataBlock's encode/decode (ida.cpp:59-162).
namespace ida {
// Fragments of one value: n rows of ceil(len / m) values (fragment i has index i + 1).
inline std::vector<std::vector<uint16_t>> Encode(const std::string &value, int n = 14, int m = 10,
                                                 int p = 257, int device = 0) {
    const uint64_t offs[2] = {0, value.size()};
    uint64_t seg[2];
    check(cx_ida_segments(offs, 1, m, seg));
    const size_t S = seg[1];
    std::vector<uint16_t> flat(n * S + 1);
    check(cx_ida_encode(reinterpret_cast<const uint8_t *>(value.data()), offs, seg, 1, n, m, p,
                        flat.data(), CX_MEM_HOST, device));
    std::vector<std::vector<uint16_t>> rows(n);
    for (int i = 0; i < n; ++i) rows[i].assign(flat.begin() + i * S, flat.begin() + (i + 1) * S);
    return rows;
}

// IDA::Decode from m fragments (index, values), trailing zeros dropped;
// throws "N is not invertible" like matrix_math.cpp:81-82.
inline std::vector<uint16_t> Decode(const std::vector<std::pair<int, std::vector<uint16_t>>> &frags,
                                    int m = 10, int p = 257, int device = 0) {
    if ((int)frags.size() < m)
        throw Error(CX_E_INSUFFICIENT, std::to_string(m) + " frags are required to decode.");
    const size_t S = frags[0].second.size();
    std::vector<uint16_t> flat;
    std::vector<uint8_t> idx;
    for (int k = 0; k < m; ++k) {
        flat.insert(flat.end(), frags[k].second.begin(), frags[k].second.end());
        idx.push_back((uint8_t)frags[k].first);
    }
    flat.push_back(0);
    const uint64_t seg[2] = {0, S};
    std::vector<uint16_t> out(m * S + 1);
    uint64_t len = 0;
    check(cx_ida_decode(flat.data(), seg, idx.data(), 1, m, p, out.data(), &len, CX_MEM_HOST,
                        device));
    if (len == UINT64_MAX) throw Error(CX_E_INVALID, "N is not invertible");
    out.resize(len);
    return out;
}
}  // namespace ida

}  // namespace chordx
