// test_chordx_api.cpp -- the reference's gtest cases for the lookup path,
// re-expressed against include/chordx.hpp (runs on the GPU; driven by
// tests/test_cpp_api.py).  Fixture values come from tests/golden/
// reference_vectors.json (test/test_json/** and test/key_test.cc data).
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/chordx.hpp"

static int failures = 0;
#define EXPECT_TRUE(c) do { if (!(c)) { ++failures; std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); } } while (0)
#define EXPECT_FALSE(c) EXPECT_TRUE(!(c))
#define EXPECT_EQ(a, b) EXPECT_TRUE((a) == (b))
#define TEST(suite, name) static void suite##_##name()
#define RUN(suite, name) do { suite##_##name(); std::printf("[ RUN ] %s.%s\n", #suite, #name); } while (0)

using chordx::Key;
using chordx::Ring;

TEST(KeyInBetweenTest, ExclusiveNoModulo) {
    EXPECT_TRUE(Key(0, 75).InBetween(Key(0, 0), Key(0, 99), false));
    EXPECT_FALSE(Key(0, 99).InBetween(Key(0, 0), Key(0, 99), false));
}
TEST(KeyInBetweenTest, ExclusiveWithModulo) {
    EXPECT_TRUE(Key(0, 1).InBetween(Key(0, 75), Key(0, 25), false));
    EXPECT_FALSE(Key(0, 25).InBetween(Key(0, 75), Key(0, 25), false));
}
TEST(KeyInBetweenTest, InclusiveNoModulo) {
    EXPECT_TRUE(Key(0, 75).InBetween(Key(0, 0), Key(0, 99), true));
    EXPECT_TRUE(Key(0, 99).InBetween(Key(0, 0), Key(0, 99), true));
}
TEST(KeyInBetweenTest, InclusiveWithModulo) {
    EXPECT_TRUE(Key(0, 1).InBetween(Key(0, 75), Key(0, 25), true));
    EXPECT_TRUE(Key(0, 25).InBetween(Key(0, 75), Key(0, 25), true));
}
TEST(KeyInBetweenTest, DifferingLengths) {
    Key key = Key::FromHex("f4ee136cb4059b2883450e7e93698be"),
        lb = Key::FromHex("633bd46b5c515992a5ce553d0680bec9"),
        ub = Key::FromHex("f4ee136cb4059b2883450e7e93698bd");
    EXPECT_FALSE(key.InBetween(lb, ub, true));
    EXPECT_EQ(key.Str(), std::string("f4ee136cb4059b2883450e7e93698be"));
}

TEST(ChordIntegration, Join) {
    const char *peers[] = {
        "36a22c462b875f71b5bad53d1909761d",
        "633bd46b5c515992a5ce553d0680bec8",
        "94227b6ddb5a5ee68a4b8c7627640f5d",
        "ad8bf45ee3435094b624b513fdb21c1d",
        "b9c49b7b7a18545e924cf36f8b9d3afd",
        "e2a708de118a51bf948e9320eeac848c"};
    struct { const char *key, *owner; } kv[] = {
        {"ed7e9a11fb0b56d58fe3aab83e01dff2", "36a22c462b875f71b5bad53d1909761d"},
        {"f02f9a33a1325add82c9f2935627fde8", "36a22c462b875f71b5bad53d1909761d"},
        {"ad40ad8bebe5093bd9ea7a252b372b0", "36a22c462b875f71b5bad53d1909761d"},
        {"21c6b801af4458738a829ee4726f14c0", "36a22c462b875f71b5bad53d1909761d"},
        {"4d1f65d6a4af5419a51f6406aa23a2bf", "633bd46b5c515992a5ce553d0680bec8"},
        {"8f218246f4e35dc7b60419ff9fcbce73", "94227b6ddb5a5ee68a4b8c7627640f5d"},
        {"a81fd109d24757e39fcb2fb9ab345672", "ad8bf45ee3435094b624b513fdb21c1d"},
        {"a8f274ce76875f48b20ff0fa1d9e3941", "ad8bf45ee3435094b624b513fdb21c1d"},
        {"da9c4c9382605ae289c62a51f14a7949", "e2a708de118a51bf948e9320eeac848c"},
        {"db8d652ed2e7541ea8034f2603232d64", "e2a708de118a51bf948e9320eeac848c"}};
    std::vector<Key> ids;
    for (const char *p : peers) ids.push_back(Key::FromHex(p));
    Ring ring(ids);
    ring.PopulateFingerTable();
    std::vector<Key> all = ring.Ids();
    const uint32_t src = ring.IndexOf(ids[0]);  // keys are created from peers[0]
    for (const auto &e : kv) {
        chordx::Lookup l = ring.GetSuccessor(src, Key::FromHex(e.key));
        EXPECT_EQ(all[l.owner].Str(), std::string(e.owner));
        EXPECT_EQ(all[ring.Owner(Key::FromHex(e.key))].Str(), std::string(e.owner));
    }
}

TEST(ChordGetSucc, FromFingerTable) {
    Ring ring({Key::FromHex("62a0959bff135ad296fbdc29252d927a"), Key::FromHex("5c22f4050c375657b05b35732eef0130")});
    ring.PopulateFingerTable();
    chordx::Lookup l = ring.GetSuccessor(ring.IndexOf(Key::FromHex("62a0959bff135ad296fbdc29252d927a")),
                                         Key::FromHex("62a0959bff135ad296fbdc29252d927b"));
    EXPECT_EQ(ring.Ids()[l.owner].Str(), std::string("5c22f4050c375657b05b35732eef0130"));
    EXPECT_EQ(l.hops, 1);
}

// ChordGetPred.InSuccList / FromFingerTable (chord_test.cpp:131-227,
// GetPredTest.json): the converged answer, batched.
TEST(ChordGetPred, Fixtures) {
    Ring a({Key::FromHex("8fcd40610a285f29ad7168be553d20db"),
            Key::FromHex("f7ad227bcc0f55b3b15927475dd5a053"),
            Key::FromHex("67cd3c64a95a51229cf89ec7a252772a")});
    EXPECT_EQ(a.Ids()[a.GetPredecessor(Key::FromHex("67cd3c64a95a51229cf89ec7a2527729"))].Str(),
              std::string("f7ad227bcc0f55b3b15927475dd5a053"));
    Ring b({Key::FromHex("459a8765538b59a2b2a046143026ed56"),
            Key::FromHex("3b74d34668f5258974b09b496fa4bb0")});
    EXPECT_EQ(b.Ids()[b.GetPredecessor(Key::FromHex("459a8765538b59a2b2a046143026ed57"))].Str(),
              std::string("459a8765538b59a2b2a046143026ed56"));
}

TEST(ChordGetSucc, FromPredecessor) {
    Ring ring({Key::FromHex("61b23792c54457c5ac5b7a95b35722db"), Key::FromHex("f56febc96cfa5a6f8469b933a76dd0e0")});
    std::vector<uint32_t> F = ring.FingerTable();
    const uint32_t s = ring.IndexOf(Key::FromHex("61b23792c54457c5ac5b7a95b35722db"));
    for (unsigned i = 0; i < CX_FINGERS; ++i) F[s * CX_FINGERS + i] = s;  // AdjustFingers(self)
    ring.EditFingers(F);
    chordx::Lookup l = ring.GetSuccessor(s, Key::FromHex("61b23792c54457c5ac5b7a95b35722dc"));
    EXPECT_EQ(l.owner, 1 - s);  // the predecessor
    EXPECT_EQ(l.hops, 1);
}

// StoredLocally for a batch (abstract_chord_peer.cpp:720-725), through the
// C++ mirror: a 4 096-peer ring and 2^16 + 3 x 512 keys (so the engine takes
// its LDS slice table) against the first ID >= key with wrap, on the host.
TEST(ChordStoredLocally, Batch) {
    auto mix = [](uint64_t x) {
        x += 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        return x ^ (x >> 31);
    };
    std::vector<Key> ids;
    for (uint64_t i = 0; i < 4096; ++i) ids.push_back(Key(mix(2 * i), mix(2 * i + 1)));
    Ring ring(ids);
    const std::vector<Key> sorted = ring.Ids();
    std::vector<Key> keys;
    for (uint64_t i = 0; i < (1u << 16); ++i) keys.push_back(Key(mix(1000003 + 2 * i), mix(1000004 + 2 * i)));
    for (size_t j = 0; j < 512; ++j) {  // an ID, its neighbours
        const unsigned __int128 v = sorted[j * 8].value();
        keys.push_back(Key(v));
        keys.push_back(Key(v + 1));
        keys.push_back(Key(v - 1));
    }
    const std::vector<uint32_t> got = ring.Successors(keys);
    size_t bad = 0;
    for (size_t i = 0; i < keys.size(); ++i) {
        size_t a = 0, z = sorted.size();
        while (a < z) {
            const size_t m = (a + z) / 2;
            if (sorted[m] < keys[i]) a = m + 1;
            else z = m;
        }
        bad += got[i] != (a == sorted.size() ? 0u : (uint32_t)a);
    }
    EXPECT_EQ(bad, (size_t)0);
}

// GET_SUCC_FAILING (GetSuccTest.json): peer 127.0.0.1:7003 (constructed, its
// server answers, min_key_ = id_, StartChord never called -> empty finger
// table); its predecessor_ and only successor are a peer with ID
// fff...f (31 f) on port 1 that never answers.  EXPECT_ANY_THROW.
static std::string failing_throw(bool fill_fingers, int rule) {
    const Key p = Key::FromHex("61b23792c54457c5ac5b7a95b35722db");  // UUIDv5("127.0.0.1:7003")
    const Key dead = Key::FromHex("fffffffffffffffffffffffffffffff");
    Ring ring({p, dead});
    const uint32_t ip = ring.IndexOf(p), id = ring.IndexOf(dead);
    std::vector<uint32_t> F(2 * CX_FINGERS, CX_NONE);  // empty table: no finger added
    if (fill_fingers)  // what the test's comment intends AdjustFingers(succ) to do
        for (unsigned i = 0; i < CX_FINGERS; ++i) F[ip * CX_FINGERS + i] = id;
    ring.EditFingers(F);
    std::vector<Key> mk(2);
    mk[ip] = p;                       // min_key_(id_), abstract_chord_peer.cpp:22
    mk[id] = Key::FromHex("0");       // the fixture's MIN_KEY
    std::vector<uint32_t> preds(2, CX_NONE);
    preds[ip] = id;                   // predecessor_.Set(succ)
    ring.SetPeerState(&mk, &preds);
    std::vector<uint8_t> alive(2, 0);
    alive[ip] = 1;                    // port 1 never answers
    std::vector<uint32_t> succs(2 * 3, CX_NONE);
    succs[ip * 3] = id;               // successors_.Insert(succ)
    ring.SetLiveness(&alive, &succs, 3, rule);
    try {
        ring.GetSuccessor(ip, Key::FromHex("0000000000000000000000000000000"));
    } catch (const chordx::Error &e) {
        return e.what();
    }
    return "";
}

TEST(ChordGetSucc, Failing) {
    // literal: FingerTable::Lookup over the empty table throws (finger_table.h:129)
    EXPECT_EQ(failing_throw(false, CX_FWD_CHORD), std::string("ChordKey not found"));
    // every finger = the dead succ: successors_.Lookup -> dead -> chord_peer.cpp:206
    EXPECT_EQ(failing_throw(true, CX_FWD_CHORD), std::string("Lookup failed"));
    // DHash rule: LookupLiving none, successors_[0] dead -> dhash_peer.cpp:524
    EXPECT_EQ(failing_throw(true, CX_FWD_DHASH), std::string("Lookup failed"));
}

TEST(ChordGetSucc, LivelockHitsHopCap) {
    // every finger points at the peer itself and its predecessor is unset: the
    // reference forwards to itself forever; chordx stops at the hop cap
    Ring ring({Key::FromHex("62a0959bff135ad296fbdc29252d927a"), Key::FromHex("5c22f4050c375657b05b35732eef0130")});
    std::vector<uint32_t> F = ring.FingerTable();
    for (unsigned i = 0; i < CX_FINGERS; ++i) F[i] = 0;
    ring.EditFingers(F);
    std::vector<uint32_t> preds = {CX_NONE, 0};
    ring.SetPeerState(nullptr, &preds);
    chordx::Lookup l = ring.Route({0}, {Key(ring.Ids()[1].value())})[0];
    EXPECT_EQ(l.status, CX_Q_HOPCAP);
    EXPECT_EQ(l.hops, CX_HOP_CAP);
}

TEST(DHashPeer, InsufficientSuccs) {
    std::vector<Key> ids;
    for (int i = 0; i < 9; ++i) ids.push_back(Key(0x1000ull * i, 7));
    Ring ring(ids);
    bool threw = false;
    try {
        ring.CheckReplicas(14, 10);
    } catch (const chordx::Error &e) {
        threw = std::string(e.what()).find("Insufficient succs") == 0;
    }
    EXPECT_TRUE(threw);
    EXPECT_EQ(ring.GetNSuccessors(Key(0, 5), 14).size(), 9u);
}

TEST(Wire, GetSuccJoinFixture) {
    // ChordIntegration.Join peers by name; key1 belongs to 94227b6d... (port 5003)
    chordx::Wire w({"127.0.0.1:5000", "127.0.0.1:5001", "127.0.0.1:5002", "127.0.0.1:5003",
                    "127.0.0.1:5004", "127.0.0.1:5005"});
    const std::string r = w.Handle("{\"COMMAND\":\"GET_SUCC\",\"KEY\":\"8f218246f4e35dc7b60419ff9fcbce73\"}");
    EXPECT_TRUE(r.find("\"ID\":\"94227b6ddb5a5ee68a4b8c7627640f5d\"") != std::string::npos);
    EXPECT_TRUE(r.find("\"PORT\":5003") != std::string::npos);
    EXPECT_TRUE(r.find("\"SUCCESS\":true") != std::string::npos);
    const std::string bad = w.Handle("{\"COMMAND\":\"NOPE\"}");
    EXPECT_TRUE(bad.find("Invalid command.") != std::string::npos);
}

TEST(DataBlock, EncodeDecodeVal1) {
    // DHashIntegration.CreateAndRead stores "val1" (dhash_test.cpp:213-226)
    const std::string v = "val1";
    auto rows = chordx::ida::Encode(v);
    EXPECT_EQ(rows.size(), 14u);
    std::vector<std::pair<int, std::vector<uint16_t>>> alive;
    for (int i : {1, 2, 4, 5, 6, 8, 9, 10, 12, 13}) alive.push_back({i + 1, rows[i]});
    std::vector<uint16_t> back = chordx::ida::Decode(alive);
    EXPECT_EQ(std::string(back.begin(), back.end()), v);
    bool threw = false;
    alive[1].first = alive[0].first;  // repeated index
    try {
        const std::vector<uint16_t> got = chordx::ida::Decode(alive);
        std::printf("no error: decoded %zu values\n", got.size());
    } catch (const chordx::Error &e) {
        threw = std::string(e.what()) == "N is not invertible";
        if (!threw) std::printf("unexpected error: %s\n", e.what());
    }
    EXPECT_TRUE(threw);
}

int main() {
    RUN(KeyInBetweenTest, ExclusiveNoModulo);
    RUN(KeyInBetweenTest, ExclusiveWithModulo);
    RUN(KeyInBetweenTest, InclusiveNoModulo);
    RUN(KeyInBetweenTest, InclusiveWithModulo);
    RUN(KeyInBetweenTest, DifferingLengths);
    RUN(ChordIntegration, Join);
    RUN(ChordGetSucc, FromFingerTable);
    RUN(ChordGetSucc, FromPredecessor);
    RUN(ChordGetSucc, Failing);
    RUN(ChordGetSucc, LivelockHitsHopCap);
    RUN(ChordGetPred, Fixtures);
    RUN(ChordStoredLocally, Batch);
    RUN(DHashPeer, InsufficientSuccs);
    RUN(Wire, GetSuccJoinFixture);
    RUN(DataBlock, EncodeDecodeVal1);
    std::printf(failures ? "FAILED (%d)\n" : "PASSED\n", failures);
    return failures ? 1 : 0;
}
