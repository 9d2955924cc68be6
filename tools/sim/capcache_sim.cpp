// Analysis: would a per-batch cache of capacity upper bounds end the failing long walks of fragmented shards early?
// First-pass model of the engine: every chunk speculates against the state at its start; a maxConcurrent == 1 lane of
// rank r (its index among the chunk's lanes of its action) with memory m walks the whole pool and falls back when the
// pool's capacity C_m = sum over usable x of floor(P[x] / m) is <= r.  Today the engine skips such a walk only when
// m > U (the largest usable permit count, exact at the batch start, tightened to m - 1 after a failed rank-0 walk).
// The cache: a failed walk (mem m, capacity T) proves C_m' <= T for every m' >= m for the rest of the batch (permits
// only fall inside a batch), so a later lane of rank r >= T with mem >= m falls back without walking.
//   g++ -O2 -o /tmp/capsim tools/sim/capcache_sim.cpp && /tmp/capsim /tmp/sim/headline_of8 192
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>
using namespace std;
template <class T> vector<T> load(const string& d, const char* n) {
    string p = d + "/" + n + ".bin";
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) { perror(p.c_str()); exit(1); }
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    vector<T> v(sz / sizeof(T)); if (fread(v.data(), 1, sz, f) != (size_t)sz) exit(1); fclose(f); return v;
}
int main(int argc, char** argv) {
    string d = argv[1];
    const int CW = argc > 2 ? atoi(argv[2]) : 192;
    auto perm = load<int32_t>(d, "perm"), mpool = load<int32_t>(d, "mpool"), bpool = load<int32_t>(d, "bpool"),
         usable = load<int32_t>(d, "usable"), mem = load<int32_t>(d, "mem"), maxc = load<int32_t>(d, "maxc"),
         pool = load<int32_t>(d, "pool"), act = load<int32_t>(d, "act"), out = load<int32_t>(d, "out"),
         slot = load<int32_t>(d, "slot");
    auto acq_off = load<int64_t>(d, "acq_off"), rel_off = load<int64_t>(d, "rel_off"), rel_aid = load<int64_t>(d, "rel_aid");
    vector<int32_t> P = perm;
    unordered_map<long, pair<int, int>> cm;
    const int NB = acq_off.size() - 1;
    long walks_today = 0, walks_cache = 0, steps_today = 0, steps_cache = 0, fb_mc1 = 0, skipped_U = 0;
    for (int b = 0; b < NB; ++b) {
        for (int64_t r = rel_off[b]; r < rel_off[b + 1]; ++r) {
            int64_t aid = rel_aid[r]; int a = act[aid], x = out[aid];
            if (x < 0) continue;
            if (maxc[a] == 1) { P[x] += mem[a]; continue; }
            auto& e = cm[(long)x << 20 | slot[a]];
            e.second--; int n2 = e.first + 1;
            if (n2 % maxc[a] == 0) { e.first = n2 - maxc[a]; P[x] += mem[a]; } else e.first = n2;
            if (e.second == 0) cm.erase((long)x << 20 | slot[a]);
        }
        int U[2];
        for (int p = 0; p < 2; ++p) { U[p] = -1; for (int y : (p ? bpool : mpool)) if (usable[y]) U[p] = max(U[p], P[y]); }
        map<int, long> cache[2];  // mem -> capacity upper bound (valid for every mem' >= mem)
        for (int64_t c0 = acq_off[b]; c0 < acq_off[b + 1]; c0 += CW) {
            const int64_t end = min(c0 + CW, acq_off[b + 1]);
            unordered_map<int, int> rank;
            map<pair<int, int>, long> capm;  // (pool, mem) -> C at the chunk start
            vector<pair<int, long>> fails[2];
            auto cap_of = [&](int p, int m) {
                auto k = make_pair(p, m);
                auto it = capm.find(k);
                if (it != capm.end()) return it->second;
                long C = 0;
                for (int y : (p ? bpool : mpool)) if (usable[y] && P[y] >= m) C += P[y] / m;
                capm[k] = C;
                return C;
            };
            for (int64_t i = c0; i < end; ++i) {
                const int a = act[i];
                const int r = rank[a]++;
                if (maxc[a] != 1) continue;
                const int p = pool[a], m = mem[a];
                const int n = (p ? bpool : mpool).size();
                if (out[i] >= 0 && true) {
                    // decided by a placement: a walk that fails in the first pass is still possible (rank r beyond the
                    // chunk-start capacity while earlier lanes go elsewhere) -- counted below through C
                }
                if (m > U[p]) { ++skipped_U; continue; }
                const long C = cap_of(p, m);
                if (C > r) continue;  // the first-pass walk finds a target
                ++fb_mc1;
                ++walks_today;
                steps_today += n;
                bool hit = false;
                for (auto& kv : cache[p]) {
                    if (kv.first > m) break;
                    if (kv.second <= r) { hit = true; break; }
                }
                if (!hit) { ++walks_cache; steps_cache += n; fails[p].push_back({m, C}); }
                if (r == 0) U[p] = min(U[p], m - 1);
            }
            for (int p = 0; p < 2; ++p)
                for (auto& f : fails[p]) {
                    auto it = cache[p].find(f.first);
                    if (it == cache[p].end() || it->second > f.second) cache[p][f.first] = f.second;
                }
            // apply the chunk's decisions
            for (int64_t i = c0; i < end; ++i) {
                const int a = act[i], x = out[i];
                if (x < 0) continue;
                if (maxc[a] == 1) { P[x] -= mem[a]; continue; }
                auto& e = cm[(long)x << 20 | slot[a]];
                if (e.first >= 1) { e.first--; e.second++; }
                else { P[x] -= mem[a]; e.second++; int n2 = e.first + maxc[a] - 1; e.first = (n2 % maxc[a] == 0) ? n2 - maxc[a] : n2; }
            }
        }
    }
    printf("%s cw %d: first-pass failing long walks %ld (%ld pool steps); with the capacity cache %ld (%ld steps); "
           "lanes skipped by U %ld\n", d.c_str(), CW, walks_today, steps_today, walks_cache, steps_cache, skipped_U);
}
