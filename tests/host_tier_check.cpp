// host_tier_check.cpp -- CPU differential test of the host tier after batches (host_tier.hpp,
// host_delta.hpp).  A tier that holds a base copy plus every later batch folded into its delta tree
// must answer every question -- rank, select, rank-range and key-bound aggregates, key dumps, whole
// protocol rounds -- exactly as a tier rebuilt from the merged contents (the full refresh it
// replaces).  The model is a std::map folded with the reference's semantics: insert-or-overwrite
// replaces the element's fingerprint, remove drops it (rsos/src/fingerprint_tree_map/mutate.rs:23-154).
//
//   host_tier_check <key_kind 0|1|2 (u32 | u64 | bytes16)> <seed> <base> <universe> <batches> <batch_max>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "../reconcile-rs_amd/csrc/host_tier.hpp"

using rh::DeltaTree;
using rh::HostTier;

static int failures = 0;
#define EXPECT(cond, ...)                                  \
    do {                                                   \
        if (!(cond)) {                                     \
            if (failures++ < 20) {                         \
                fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
                fprintf(stderr, __VA_ARGS__);              \
                fprintf(stderr, "\n");                     \
            }                                              \
        }                                                  \
    } while (0)

struct Fp {
    uint64_t w[4];
};

int main(int argc, char **argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: host_tier_check <kind> <seed> <base> <universe> <batches> <batch_max>\n");
        return 2;
    }
    const int kind = atoi(argv[1]);
    const uint64_t seed = strtoull(argv[2], nullptr, 10), nbase = strtoull(argv[3], nullptr, 10),
                   universe = strtoull(argv[4], nullptr, 10), batches = strtoull(argv[5], nullptr, 10),
                   batch_max = strtoull(argv[6], nullptr, 10);
    const int kk = kind == 0 ? RH_KEY_U32 : kind == 1 ? RH_KEY_U64 : RH_KEY_BYTES;
    const uint32_t kl = kind == 0 ? 4 : kind == 1 ? 8 : 16;
    rh::KeyOrder ko{kl, kk};
    std::mt19937_64 rng(seed);

    // the key universe: distinct keys; byte keys share leading bytes often (ties past the digit)
    std::vector<std::string> uni;
    {
        std::map<std::string, int, std::function<bool(const std::string &, const std::string &)>> seen(
            [&](const std::string &a, const std::string &b) {
                return ko.cmp((const uint8_t *)a.data(), (const uint8_t *)b.data()) < 0;
            });
        while (uni.size() < universe) {
            std::string k(kl, '\0');
            uint64_t x = rng();
            if (kind == 0) x %= 4 * universe + 7;
            memcpy(&k[0], &x, std::min<uint32_t>(kl, 8));
            if (kl > 8) {
                if (rng() % 3 == 0) memset(&k[0], 0x5a, 8);  // a shared leading digit
                uint64_t y = rng();
                memcpy(&k[8], &y, 8);
            }
            if (seen.emplace(k, 0).second) uni.push_back(k);
        }
    }
    auto less = [&](const std::string &a, const std::string &b) {
        return ko.cmp((const uint8_t *)a.data(), (const uint8_t *)b.data()) < 0;
    };
    std::map<std::string, Fp, decltype(less)> model(less);
    auto rand_fp = [&]() {
        Fp f;
        for (auto &w : f.w) w = rng();
        if (rng() % 8 == 0) f.w[0] = f.w[1] = f.w[2] = f.w[3] = ~0ull;  // carries through every limb
        return f;
    };
    std::shuffle(uni.begin(), uni.end(), rng);
    for (uint64_t i = 0; i < nbase && i < uni.size(); i++) model.emplace(uni[i], rand_fp());

    // a plain tier over the model's contents (what a full refresh would copy down)
    struct Flat {
        std::vector<uint8_t> keys;
        std::vector<uint64_t> prefix;
    };
    auto flatten = [&](Flat &f) {
        f.keys.clear();
        f.prefix.assign(4, 0);
        uint64_t acc[4] = {0, 0, 0, 0};
        for (auto &kv : model) {
            f.keys.insert(f.keys.end(), kv.first.begin(), kv.first.end());
            rh::fp4_add(acc, kv.second.w);
            f.prefix.insert(f.prefix.end(), acc, acc + 4);
        }
        f.keys.resize(f.keys.size() + 64);
    };
    Flat base, cur;
    flatten(base);
    HostTier A;
    A.build(kl, kk, model.size(), base.keys.data(), base.prefix.data());
    // A run copy (HostTier::Run): every key whose state differs from A's base copy, with the
    // device's DeltaRec rule (contrib = cur - base, count delta = live - in_base) and prefix sums
    struct RunArrays {
        std::vector<uint8_t> keys, flags;
        std::vector<uint64_t> prefix, samp, samp2, gsamp;
        std::vector<int32_t> cntp;
        std::vector<uint32_t> brank;
    } run;
    auto take_run = [&](bool with_index) {
        run = RunArrays{};
        const uint64_t nbase = A.nb;
        auto base_key = [&](uint64_t i) { return std::string((const char *)base.keys.data() + i * kl, kl); };
        auto base_fp = [&](uint64_t i, uint64_t out[4]) {
            memcpy(out, &base.prefix[4 * (i + 1)], 32);
            rh::fp4_sub(out, &base.prefix[4 * i]);
        };
        uint64_t acc[4] = {0, 0, 0, 0};
        int32_t cacc = 0;
        run.prefix.assign(4, 0);
        run.cntp.push_back(0);
        auto emit = [&](const std::string &k, uint64_t br, bool inb, bool live, const uint64_t *cur, const uint64_t *bfp) {
            uint64_t c[4] = {0, 0, 0, 0};
            if (live) memcpy(c, cur, 32);
            if (inb) rh::fp4_sub(c, bfp);
            run.keys.insert(run.keys.end(), k.begin(), k.end());
            run.flags.push_back((uint8_t)((inb ? 1 : 0) | (live ? 2 : 0)));
            run.brank.push_back((uint32_t)br);
            rh::fp4_add(acc, c);
            run.prefix.insert(run.prefix.end(), acc, acc + 4);
            cacc += (live ? 1 : 0) - (inb ? 1 : 0);
            run.cntp.push_back(cacc);
        };
        uint64_t i = 0;
        auto it = model.begin();
        while (i < nbase || it != model.end()) {
            const int c = i >= nbase ? 1 : it == model.end() ? -1 : ko.cmp(base.keys.data() + i * kl, (const uint8_t *)it->first.data());
            uint64_t bfp[4];
            if (c < 0) {  // a base key the model no longer holds: deleted
                base_fp(i, bfp);
                emit(base_key(i), i, true, false, nullptr, bfp);
                i++;
            } else if (c > 0) {  // inserted
                emit(it->first, i, false, true, it->second.w, nullptr);
                ++it;
            } else {  // in both: an entry only if the fingerprint changed
                base_fp(i, bfp);
                if (memcmp(bfp, it->second.w, 32)) emit(it->first, i, true, true, it->second.w, bfp);
                i++, ++it;
            }
        }
        const uint64_t nr = run.flags.size();
        for (uint64_t j = 0; j < nr; j += 64) run.samp.push_back(ko.digit(run.keys.data() + j * kl));
        for (uint64_t j = 0; j < nr; j += 4096) run.samp2.push_back(ko.digit(run.keys.data() + j * kl));
        for (uint64_t j = 0; j < nr; j += 64)  // select's index, as the device forms it
            run.gsamp.push_back((uint64_t)((int64_t)run.brank[j] + run.cntp[j] + ((run.flags[j] & 2) ? 1 : 0)));
        run.keys.resize(run.keys.size() + 64);
        HostTier::Run r;
        r.n = nr;
        r.keys = run.keys.data();
        r.prefix = run.prefix.data();
        r.cntp = run.cntp.data();
        r.flags = run.flags.data();
        r.brank = run.brank.data();
        r.samp = run.samp.data();
        r.samp2 = run.samp2.data();
        r.gsamp = with_index ? run.gsamp.data() : nullptr;  // with and without select's index
        A.set_run(r);
    };

    uint64_t checked = 0;
    for (uint64_t it = 0; it < batches; it++) {
        // one batch: distinct keys, sorted, ~70 % upserts (new or overwrite), ~30 % deletes
        const uint64_t m = 1 + rng() % batch_max;
        std::vector<std::string> bk;
        for (uint64_t j = 0; j < m; j++) bk.push_back(uni[rng() % uni.size()]);
        std::sort(bk.begin(), bk.end(), less);
        bk.erase(std::unique(bk.begin(), bk.end(), [&](const std::string &a, const std::string &b) {
                     return !less(a, b) && !less(b, a);
                 }),
                 bk.end());
        std::vector<DeltaTree::Rec> rows(bk.size());
        std::vector<uint8_t> drop(bk.size());
        std::vector<Fp> fps(bk.size());
        // every 4th batch is "too large for the tree": A takes a run copy of the whole change since
        // its base copy instead of folding, and later batches fold into a tree over base + run;
        // every 11th refreshes A's base (a compaction and a copy, as the store does)
        const bool snap = it % 4 == 2;
        if (it % 11 == 10) {
            flatten(base);
            A.build(kl, kk, model.size(), base.keys.data(), base.prefix.data());
        }
        for (size_t j = 0; j < bk.size(); j++) {
            const bool del = rng() % 10 < 3;
            fps[j] = rand_fp();
            drop[j] = A.entry_vs_base((const uint8_t *)bk[j].data(), del ? nullptr : fps[j].w, &rows[j]);
            if (del) model.erase(bk[j]);
            else model[bk[j]] = fps[j];
        }
        if (snap) take_run(it % 8 != 2);
        else A.fold(rows.data(), drop.data(), rows.size());

        flatten(cur);
        HostTier B;
        B.build(kl, kk, model.size(), cur.keys.data(), cur.prefix.data());
        EXPECT(A.n == B.n, "batch %llu: size %llu vs %llu", (unsigned long long)it, (unsigned long long)A.n,
               (unsigned long long)B.n);
        if (A.n != B.n) break;
        const uint64_t n = B.n;
        // select at every rank (small maps) or a sample
        const uint64_t step = n > 4000 ? n / 997 + 1 : 1;
        for (uint64_t r = 0; r < n; r += step) {
            const HostTier::Cur c = A.at(r);
            EXPECT(c.k && !memcmp(c.k, cur.keys.data() + r * kl, kl), "select(%llu)", (unsigned long long)r);
            checked++;
        }
        // ranks and key-bound aggregates of probe keys (present, absent, both ends)
        for (int q = 0; q < 300; q++) {
            const std::string &z = uni[rng() % uni.size()];
            const uint8_t *zk = (const uint8_t *)z.data();
            EXPECT(A.rank(zk) == B.rank(zk), "rank");
            {  // and against a plain binary search of the flattened model (no samples, no index)
                uint64_t lo = 0, hi = n;
                while (lo < hi) {
                    const uint64_t mid = (lo + hi) / 2;
                    if (ko.cmp(cur.keys.data() + mid * kl, zk) < 0) lo = mid + 1;
                    else hi = mid;
                }
                EXPECT(B.rank(zk) == lo, "rank vs the model: %llu vs %llu", (unsigned long long)B.rank(zk),
                       (unsigned long long)lo);
            }
            const std::string &z2 = uni[rng() % uni.size()];
            const uint8_t *zk2 = (const uint8_t *)z2.data();
            for (int lk = 0; lk < 3; lk++)
                for (int hk = 0; hk < 3; hk++) {
                    rh_aggregate ga, gb;
                    A.agg(A.bound(lk, zk, true), A.bound(hk, zk2, false), &ga);
                    B.agg(B.bound(lk, zk, true), B.bound(hk, zk2, false), &gb);
                    EXPECT(!memcmp(&ga, &gb, sizeof ga), "bound aggregate %d %d", lk, hk);
                }
            checked += 10;
        }
        // rank-range aggregates (including hi > n and inverted) and key dumps
        for (int q = 0; q < 200; q++) {
            const uint64_t lo = rng() % (n + 3), hi = rng() % (n + 3);
            rh_aggregate ga, gb;
            A.agg(lo, hi, &ga);
            B.agg(lo, hi, &gb);
            EXPECT(!memcmp(&ga, &gb, sizeof ga), "rank aggregate [%llu, %llu)", (unsigned long long)lo,
                   (unsigned long long)hi);
            if (lo < hi && hi <= n && hi - lo <= 5000) {
                std::vector<uint8_t> ka((hi - lo) * kl), kb((hi - lo) * kl);
                A.copy_keys(lo, hi, ka.data());
                B.copy_keys(lo, hi, kb.data());
                EXPECT(ka == kb, "keys [%llu, %llu)", (unsigned long long)lo, (unsigned long long)hi);
            }
            checked++;
        }
        // whole protocol rounds: random segments with remote aggregates, some equal to the local one
        for (int policy = 0; policy < 2; policy++) {
            const size_t r = 1 + rng() % 40;
            std::vector<uint8_t> sk(r), ek(r), skeys(r * kl), ekeys(r * kl);
            std::vector<rh_aggregate> rem(r);
            for (size_t j = 0; j < r; j++) {
                sk[j] = rng() % 5 != 0;
                ek[j] = rng() % 5 != 0;
                memcpy(&skeys[j * kl], uni[rng() % uni.size()].data(), kl);
                memcpy(&ekeys[j * kl], uni[rng() % uni.size()].data(), kl);
                const HostTier::Cur a = sk[j] ? B.lt(&skeys[j * kl]) : B.begin();
                const HostTier::Cur b = ek[j] ? B.lt(&ekeys[j * kl]) : B.end();
                B.agg(a, b, &rem[j]);
                const int how = rng() % 4;
                if (how == 1) rem[j].size += 1 + rng() % 50, rem[j].fingerprint[0] ^= rng();
                else if (how == 2) rem[j] = rh_aggregate{{0, 0, 0, 0}, 0};
                else if (how == 3) rem[j].fingerprint[3] ^= 1;
            }
            rh_segments in{sk.data(), skeys.data(), ek.data(), ekeys.data(), rem.data(), r, r};
            std::vector<uint8_t> oa, ob;
            uint64_t ha[5], hb[5];
            A.round(policy, 16, in, oa, ha);
            B.round(policy, 16, in, ob, hb);
            EXPECT(oa == ob && !memcmp(ha, hb, sizeof ha), "round policy %d (%zu segments)", policy, r);
            // the batched searches (HostTier::round_batched; A holds a tree, B none) against key by key
            for (HostTier *T : {&A, &B}) {
                std::vector<uint8_t> o1, o2;
                uint64_t h1[5], h2[5];
                T->batch = true;
                T->round(policy, 16, in, o1, h1);
                T->batch = false;
                T->round(policy, 16, in, o2, h2);
                T->batch = true;
                EXPECT(o1 == o2 && !memcmp(h1, h2, sizeof h1), "batched round policy %d (%zu segments, %s)", policy, r,
                       T == &A ? "folded" : "rebuilt");
            }
            checked++;
        }
        if (failures) break;
    }
    printf("{\"ok\": %s, \"checked\": %llu, \"delta_entries\": %llu, \"run_entries\": %llu, \"size\": %llu}\n",
           failures ? "false" : "true", (unsigned long long)checked, (unsigned long long)A.dt.size(),
           (unsigned long long)A.run.n, (unsigned long long)A.n);
    return failures ? 1 : 0;
}
