// Batch-scope exact fixpoint (SURVEY.md:277-284): how many Jacobi rounds does a whole batch need?
//
// Within one batch the reference applies the batch's completions first (SCPB:327-331 via CLB:260-346), then decides the
// publishes one after another (SCPB:398-436). Permits only fall inside the batch, so decision i depends on the state
// P_i = P0 - (consumption of every decision j < i). A Jacobi round recomputes EVERY decision of the batch at once
// against the per-invoker (and, for maxConcurrent > 1, per (invoker, fqn) entry) prefix consumption of the previous
// round's assignment; the earliest decision that is not yet final becomes final every round, and a round that changes
// nothing is the sequential result (unique fixpoint). The simulator reports, per batch: rounds to the fixpoint, how
// many decisions change per round, walk steps per round, and checks the fixpoint against the oracle's assignment.
//
// Semantics followed: schedule SCPB:398-436 (n + 2 probes, usable short-circuit SCPB:413, counter-RNG fallback over the
// usable invokers in pool order SCPB:417-424), NestedSemaphore.tryAcquireConcurrent NS:57-82 (a free slot of the
// (invoker, fqn) entry first, else the action's memory opens a container holding maxConcurrent - 1 more slots),
// releases NS:98-113 / RS:42-56.
//
//   python tools/sim/dump_workload.py c2            # -> /tmp/sim/c2/*.bin
//   g++ -O2 -o /tmp/bfsim tools/sim/batch_fixpoint_sim.cpp && /tmp/bfsim /tmp/sim/c2 [guess 0|1] [window]
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>
#include <string>
#include <unordered_map>
#include <algorithm>
using namespace std;
template <class T> vector<T> load(const string& d, const char* n) {
    string p = d + "/" + n + ".bin";
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) { perror(p.c_str()); exit(1); }
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    vector<T> v(sz / sizeof(T)); if (fread(v.data(), 1, sz, f) != (size_t)sz) exit(1); fclose(f); return v;
}
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
static inline uint32_t rng_index(uint64_t seed, uint64_t seq, uint32_t n) {
    uint64_t u = splitmix64(seed ^ (seq * 0x9E3779B97F4A7C15ULL)) >> 32;
    return (uint32_t)((u * (uint64_t)n) >> 32);
}

int main(int argc, char** argv) {
    string d = argv[1];
    const int guess = argc > 2 ? atoi(argv[2]) : 1;       // 0: first step feasible at the batch start; 1: rank packing
    const long window = argc > 3 ? atol(argv[3]) : 0;      // > 0: Jacobi over windows of this many decisions in turn
    const int scanR = argc > 4 ? atoi(argv[4]) : -1;       // >= 0: exactness scan after each round, with up to scanR
                                                           // exact re-decisions per round (-1: plain Jacobi)
    long tot_redecide = 0, dmax = 0;
    auto perm = load<int32_t>(d, "perm"), mpool = load<int32_t>(d, "mpool"), bpool = load<int32_t>(d, "bpool"),
         usable = load<int32_t>(d, "usable"), home = load<int32_t>(d, "home"), step = load<int32_t>(d, "step"),
         mem = load<int32_t>(d, "mem"), maxc = load<int32_t>(d, "maxc"), pool = load<int32_t>(d, "pool"),
         act = load<int32_t>(d, "act"), out = load<int32_t>(d, "out"), slot = load<int32_t>(d, "slot");
    auto acq_off = load<int64_t>(d, "acq_off"), rel_off = load<int64_t>(d, "rel_off"), rel_aid = load<int64_t>(d, "rel_aid");
    auto seedv = load<uint64_t>(d, "seed");
    const uint64_t seed = seedv[0];
    const int NB = acq_off.size() - 1, NX = perm.size();
    vector<int32_t> hl[2];  // usable ids per pool in pool order
    for (int p = 0; p < 2; ++p)
        for (int y : (p ? bpool : mpool)) if (usable[y]) hl[p].push_back(y);
    vector<int> mems, memidx(mem.size());
    for (size_t a = 0; a < mem.size(); ++a) {
        auto it = find(mems.begin(), mems.end(), mem[a]);
        if (it == mems.end()) { memidx[a] = mems.size(); mems.push_back(mem[a]); } else memidx[a] = it - mems.begin();
    }
    const int NM = mems.size();
    vector<long> tau((size_t)perm.size() * NM);
    vector<int32_t> P = perm;
    unordered_map<long, pair<int, int>> cm;  // (x, slot) -> (free c, ops)
    auto ckey = [](int x, int s) { return (long)x << 20 | s; };
    vector<int> rounds_per_batch;
    long tot_rounds = 0, tot_dec = 0, tot_changes = 0, tot_steps = 0, tot_recomp = 0;
    vector<long> changes_by_round(4096, 0), active_by_round(4096, 0);
    int maxr = 0;
    for (int b = 0; b < NB; ++b) {
        for (int64_t r = rel_off[b]; r < rel_off[b + 1]; ++r) {
            int64_t aid = rel_aid[r]; int a = act[aid], x = out[aid];
            if (x < 0) continue;
            if (maxc[a] == 1) { P[x] += mem[a]; continue; }
            auto it = cm.find(ckey(x, slot[a]));
            if (it == cm.end()) continue;
            auto& e = it->second;
            e.second--; int n2 = e.first + 1;
            if (n2 % maxc[a] == 0) { e.first = n2 - maxc[a]; P[x] += mem[a]; } else e.first = n2;
            if (e.second == 0) cm.erase(it);
        }
        const int64_t a0 = acq_off[b], a1 = acq_off[b + 1];
        const long B = a1 - a0;
        if (!B) continue;
        // static start of each walk: the first step feasible against the batch-start state (permits only fall, a free
        // slot only disappears once taken: a step infeasible at the start stays infeasible for the whole batch)
        vector<int> start(B), tgt(B), ntgt(B);
        auto walk = [&](long k, auto&& feasible, long& steps) -> int {  // returns the target id (fallback: RNG pick)
            const int a = act[a0 + k];
            const vector<int32_t>& pl = pool[a] ? bpool : mpool;
            const int n = pl.size();
            long pos = (home[a] + (long)start[k] * step[a]) % n;
            for (int s = start[k]; s < n + 2; ++s) {
                ++steps;
                int y = pl[pos];
                if (usable[y] && feasible(y)) return y;
                pos += step[a]; if (pos >= n) pos -= n;
            }
            const auto& H = hl[pool[a]];
            if (H.empty()) return -1;
            return H[rng_index(seed, (uint64_t)(a0 + k), H.size())];
        };
        {
            long dummy = 0;
            for (long k = 0; k < B; ++k) {
                start[k] = 0;
                const int a = act[a0 + k];
                const vector<int32_t>& pl = pool[a] ? bpool : mpool;
                const int n = pl.size();
                long pos = home[a] % n; int s = 0;
                for (; s < n + 2; ++s) {
                    int y = pl[pos];
                    if (usable[y]) {
                        if (P[y] >= mem[a]) break;
                        if (maxc[a] > 1) { auto it = cm.find(ckey(y, slot[a])); if (it != cm.end() && it->second.first >= 1) break; }
                    }
                    pos += step[a]; if (pos >= n) pos -= n;
                }
                start[k] = s;
            }
            (void)dummy;
        }
        // initial guess
        if (guess == 0) {
            for (long k = 0; k < B; ++k) {
                long st = 0; const int a = act[a0 + k];
                tgt[k] = walk(k, [&](int y) {
                    if (P[y] >= mem[a]) return true;
                    if (maxc[a] > 1) { auto it = cm.find(ckey(y, slot[a])); if (it != cm.end() && it->second.first >= 1) return true; }
                    return false; }, st);
            }
        } else {
            // rank packing: the r-th decision of an action in the batch skips the capacity its r predecessors take
            unordered_map<int, int> rank;
            for (long k = 0; k < B; ++k) {
                const int a = act[a0 + k];
                int r = rank[a]++;
                const vector<int32_t>& pl = pool[a] ? bpool : mpool;
                const int n = pl.size();
                long pos = (home[a] + (long)start[k] * step[a]) % n; long cum = 0; int t = -2;
                for (int s = start[k]; s < n + 2; ++s) {
                    int y = pl[pos];
                    if (usable[y]) {
                        long cap = P[y] >= mem[a] ? P[y] / mem[a] : 0;
                        if (maxc[a] > 1) {
                            cap *= maxc[a];
                            auto it = cm.find(ckey(y, slot[a])); if (it != cm.end()) cap += max(0, it->second.first);
                        }
                        cum += cap;
                        if (cum > r) { t = y; break; }
                    }
                    pos += step[a]; if (pos >= n) pos -= n;
                }
                if (t == -2) { const auto& H = hl[pool[a]]; t = H.empty() ? -1 : H[rng_index(seed, (uint64_t)(a0 + k), H.size())]; }
                tgt[k] = t;
            }
        }
        // Jacobi rounds
        int rounds = 0;
        long lo = 0;  // decisions before lo are final
        const long W = window > 0 ? window : B;
        vector<int> consum(B);                      // memory taken by decision k at its target under the assignment
        vector<int> crank(B);                       // (x, key) entry state before k: free slots
        // per invoker: sorted decision indices; prefix sums of consumption
        vector<vector<long>> bk(NX);
        vector<vector<long>> bsum(NX);
        unordered_map<long, vector<long>> pk;       // (x, slot) -> decision indices in order
        while (lo < B) {
            const long hi = min(B, lo + W);
            for (;;) {
                ++rounds;
                // consumption of the current assignment (all decisions < hi)
                for (auto& v : bk) v.clear();
                for (auto& v : bsum) v.clear();
                pk.clear();
                for (long k = 0; k < hi; ++k) {
                    int x = tgt[k]; if (x < 0) continue;
                    const int a = act[a0 + k];
                    if (maxc[a] == 1) { consum[k] = mem[a]; }
                    else {
                        auto& v = pk[ckey(x, slot[a])];
                        int j = v.size(); v.push_back(k);
                        auto it = cm.find(ckey(x, slot[a]));
                        int c0 = it == cm.end() ? 0 : it->second.first;
                        // the j-th acquisition at the entry: a free slot while some are left, else it opens a container
                        int c = c0; bool opens;
                        if (j < c0) opens = false;
                        else opens = ((j - c0) % maxc[a]) == 0;
                        (void)c;
                        consum[k] = opens ? mem[a] : 0;
                    }
                    bk[x].push_back(k);
                    bsum[x].push_back((bsum[x].empty() ? 0 : bsum[x].back()) + consum[k]);
                }
                auto before = [&](int x, long k) -> long {  // consumption at x of decisions < k
                    auto& v = bk[x];
                    long idx = lower_bound(v.begin(), v.end(), k) - v.begin();
                    return idx ? bsum[x][idx - 1] : 0;
                };
                auto slots_before = [&](int x, int s, int M, long k) -> int {
                    auto it0 = cm.find(ckey(x, s));
                    int c0 = it0 == cm.end() ? 0 : it0->second.first;
                    auto it = pk.find(ckey(x, s));
                    long j = 0;
                    if (it != pk.end()) j = lower_bound(it->second.begin(), it->second.end(), k) - it->second.begin();
                    if (j < c0) return c0 - (int)j;
                    long q = (j - c0) % M;  // after the container opened at rank c0 + M*t: M - 1 - q slots
                    return q == 0 ? 0 : (int)(M - q);
                };
                // tau[x][m]: the first decision index that finds x below m MB (permits only fall inside the batch)
                #pragma omp parallel for schedule(dynamic, 64)
                for (int x = 0; x < NX; ++x) {
                    for (int mi = 0; mi < NM; ++mi) {
                        const int m = mems[mi];
                        long t = hi;
                        if (P[x] < m) t = 0;
                        else for (size_t q = 0; q < bk[x].size(); ++q)
                            if ((long)P[x] - bsum[x][q] < m) { t = bk[x][q] + 1; break; }
                        tau[(size_t)x * NM + mi] = t;
                    }
                }
                long changes = 0, steps = 0, first_change = -1;
                #pragma omp parallel for schedule(dynamic, 256) reduction(+ : steps)
                for (long k = lo; k < hi; ++k) {
                    const int a = act[a0 + k];
                    const int mi = memidx[a];
                    ntgt[k] = walk(k, [&](int y) {
                        if (maxc[a] > 1 && slots_before(y, slot[a], maxc[a], k) >= 1) return true;
                        return k < tau[(size_t)y * NM + mi]; }, steps);
                }
                for (long k = lo; k < hi; ++k)
                    if (ntgt[k] != tgt[k]) { ++changes; if (first_change < 0) first_change = k; }
                ++tot_recomp; tot_steps += steps;
                int rr = rounds - 1; if (rr < 4096) { changes_by_round[rr] += changes; active_by_round[rr] += hi - lo; }
                tot_changes += changes;
                if (scanR >= 0 && changes) {
                    // exactness scan in stream order: ntgt[k] was computed against the OLD assignment of every j < k; it
                    // is exact when no invoker its walk looked at (steps up to its target) has a different consumption
                    // prefix under the decisions already found exact (set D). A decision whose walk touches D is
                    // re-decided exactly (up to scanR per round), else the scan stops there.
                    vector<char> inD(NX, 0);
                    vector<int> Dlist;
                    vector<int> fin(hi);
                    for (long k = 0; k < lo; ++k) fin[k] = tgt[k];
                    long k = lo; int red = 0;
                    // exact consumption of the scanned prefix: recompute on demand at D invokers from fin[]
                    auto exact_walk = [&](long kk) -> int {
                        // sequential truth for kk given fin[0..kk)
                        const int a = act[a0 + kk];
                        long st2 = 0;
                        return walk(kk, [&](int y) {
                            long c = 0; int cnt = 0;
                            for (long j = 0; j < kk; ++j) if (fin[j] == y) {
                                const int aj = act[a0 + j];
                                if (maxc[aj] == 1) c += mem[aj];
                                else {
                                    // rank of j at its entry among fin
                                    int jr = 0; for (long q = 0; q < j; ++q) if (fin[q] == y && slot[act[a0 + q]] == slot[aj]) ++jr;
                                    auto it = cm.find(ckey(y, slot[aj])); int c0 = it == cm.end() ? 0 : it->second.first;
                                    bool opens = jr >= c0 && ((jr - c0) % maxc[aj]) == 0;
                                    if (opens) c += mem[aj];
                                }
                                if (maxc[a] > 1 && slot[act[a0 + j]] == slot[a]) ++cnt;
                            }
                            if (maxc[a] > 1) {
                                auto it = cm.find(ckey(y, slot[a])); int c0 = it == cm.end() ? 0 : it->second.first;
                                int fr = cnt < c0 ? c0 - cnt : (((cnt - c0) % maxc[a]) == 0 ? 0 : maxc[a] - (cnt - c0) % maxc[a]);
                                if (fr >= 1) return true;
                            }
                            return (long)P[y] - c >= mem[a]; }, st2);
                    };
                    for (; k < hi; ++k) {
                        const int a = act[a0 + k];
                        const vector<int32_t>& pl = pool[a] ? bpool : mpool;
                        const int n = pl.size();
                        bool touch = false;
                        if (!Dlist.empty()) {
                            long pos = (home[a] + (long)start[k] * step[a]) % n;
                            bool found = false;
                            for (int s = start[k]; s < n + 2; ++s) {
                                int y = pl[pos];
                                if (usable[y] && inD[y]) { touch = true; break; }
                                if (y == ntgt[k]) { found = true; break; }
                                pos += step[a]; if (pos >= n) pos -= n;
                            }
                            if (!found && !touch) touch = true;  // a fallback looked at every step: any D entry matters
                            if (!found && touch) {
                                // fallback: touched only if some D invoker is usable in the pool (always, conservatively)
                            }
                            if (inD[ntgt[k] < 0 ? 0 : ntgt[k]] && ntgt[k] >= 0) touch = true;
                        }
                        int v = ntgt[k];
                        if (touch) {
                            if (red >= scanR) break;
                            ++red; ++tot_redecide;
                            v = exact_walk(k);
                        }
                        fin[k] = v;
                        if (v != tgt[k]) {
                            if (tgt[k] >= 0 && !inD[tgt[k]]) { inD[tgt[k]] = 1; Dlist.push_back(tgt[k]); }
                            if (v >= 0 && !inD[v]) { inD[v] = 1; Dlist.push_back(v); }
                        }
                    }
                    dmax = max(dmax, (long)Dlist.size());
                    for (long q = lo; q < k; ++q) ntgt[q] = fin[q];
                    for (long q = lo; q < hi; ++q) tgt[q] = ntgt[q];
                    if (k >= hi) break;
                    lo = k;
                    continue;
                }
                for (long k = lo; k < hi; ++k) tgt[k] = ntgt[k];
                if (!changes) break;
                lo = first_change + 1 > lo ? first_change : lo;  // everything before the first change is final
            }
            lo = hi;
        }
        rounds_per_batch.push_back(rounds);
        fprintf(stderr, "batch %d: %ld decisions, %d rounds\n", b, B, rounds);
        tot_rounds += rounds; tot_dec += B; maxr = max(maxr, rounds);
        // check against the oracle and commit the batch
        for (long k = 0; k < B; ++k) {
            if (tgt[k] != out[a0 + k]) { fprintf(stderr, "batch %d decision %ld: fixpoint %d oracle %d\n", b, k, tgt[k], out[a0 + k]); return 2; }
            const int a = act[a0 + k], x = tgt[k];
            if (x < 0) continue;
            if (maxc[a] == 1) { P[x] -= mem[a]; continue; }
            auto& e = cm[ckey(x, slot[a])];
            if (e.first >= 1) { e.first--; e.second++; }
            else { P[x] -= mem[a]; e.second++; int n2 = e.first + maxc[a] - 1; e.first = (n2 % maxc[a] == 0) ? n2 - maxc[a] : n2; }
        }
    }
    vector<int> s = rounds_per_batch; sort(s.begin(), s.end());
    printf("%s guess %d window %ld: %d batches, %ld decisions (%.0f per batch)\n", d.c_str(), guess, window, NB, tot_dec,
           (double)tot_dec / NB);
    printf("  rounds per batch: mean %.1f p50 %d p99 %d max %d; total %ld\n", (double)tot_rounds / s.size(),
           s[s.size() / 2], s[(size_t)(s.size() * 0.99)], maxr, tot_rounds);
    printf("  walk steps per decision per round %.2f; changes %ld\n", (double)tot_steps / max(1L, tot_dec) / max(1.0, (double)tot_rounds / s.size()), tot_changes);
    printf("  scan: %ld exact re-decisions (%.1f per batch), largest D %ld\n", tot_redecide, (double)tot_redecide / NB, dmax);
    printf("  per round (summed over batches): round: changed / recomputed\n");
    for (int r = 0; r < min(maxr, 40); ++r) printf("    %2d: %ld / %ld\n", r, changes_by_round[r], active_by_round[r]);
    return 0;
}
