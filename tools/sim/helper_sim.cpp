// Analysis: how much would look-ahead helpers (other CUs speculating chunk k against the slot state published at the
// start of chunk k - L, same batch) shorten the engine's walks?  Sequential replay of maxConcurrent == 1 decisions;
// per decision the walk the engine does today (from its action's cursor) and the walk from max(cursor, helper bound),
// the helper bound being the rank-packed step against the lagged snapshot (first step whose cumulative capacity
// exceeds the lane's rank among the chunk's lanes of its action), or a proven fallback (the snapshot's whole-pool
// capacity <= rank).
//   g++ -O2 -o /tmp/hsim tools/sim/helper_sim.cpp && /tmp/hsim /tmp/sim/c2 192 2
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <string>
#include <deque>
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
int main(int argc, char** argv) {
    string d = argv[1];
    const int CW = argc > 2 ? atoi(argv[2]) : 192, L = argc > 3 ? atoi(argv[3]) : 2;
    auto perm = load<int32_t>(d, "perm"), mpool = load<int32_t>(d, "mpool"), bpool = load<int32_t>(d, "bpool"),
         usable = load<int32_t>(d, "usable"), home = load<int32_t>(d, "home"), step = load<int32_t>(d, "step"),
         mem = load<int32_t>(d, "mem"), maxc = load<int32_t>(d, "maxc"), pool = load<int32_t>(d, "pool"),
         act = load<int32_t>(d, "act"), out = load<int32_t>(d, "out"), slot = load<int32_t>(d, "slot");
    auto acq_off = load<int64_t>(d, "acq_off"), rel_off = load<int64_t>(d, "rel_off"), rel_aid = load<int64_t>(d, "rel_aid");
    // permits over time: replay the reference decisions (concurrent lanes: memory only when a container opens; tracked
    // through a per-(invoker, key) free-slot map)
    vector<int32_t> P = perm;
    unordered_map<long, pair<int, int>> cm;  // (x, slot) -> (free c, ops)
    const int NB = acq_off.size() - 1, A = home.size();
    vector<int> cur(A, 0);
    deque<vector<int32_t>> snaps;
    long eng_fb_walk = 0, eng_fb_walks = 0, cap_fb_walk = 0, cap_fb_walks = 0;
    int Ueng[2] = {0, 0};  // P at the start of the last L + 1 chunks of the batch
    long n1 = 0, long_today = 0, long_help = 0, steps_today = 0, steps_help = 0, fb_total = 0, fb_proven = 0,
         helped = 0, fb_walk_today = 0, fb_walk_help = 0;
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
        fill(cur.begin(), cur.end(), 0);
        snaps.clear();
        for (int p = 0; p < 2; ++p) { Ueng[p] = -1; for (int y : (p ? bpool : mpool)) if (usable[y]) Ueng[p] = max(Ueng[p], P[y]); }
        for (int64_t c0 = acq_off[b]; c0 < acq_off[b + 1]; c0 += CW) {
            snaps.push_back(P);
            if ((int)snaps.size() > L + 1) snaps.pop_front();
            const bool have = (int)snaps.size() == L + 1;  // chunk k - L is in this batch
            const vector<int32_t>& S = snaps.front();
            const int64_t end = min(c0 + CW, acq_off[b + 1]);
            unordered_map<int, int> rank;
            unordered_map<long, long> capm;  // (pool, mem) -> snapshot capacity
            for (int64_t i = c0; i < end; ++i) {
                const int a = act[i], x = out[i];
                const vector<int32_t>& pl = pool[a] ? bpool : mpool;
                const int n = pl.size();
                if (maxc[a] == 1) {
                    const int r = rank[a]++;
                    ++n1;
                    // true step of x on a's walk (fallbacks: n)
                    long pos = (home[a] + (long)cur[a] * step[a]) % n; int s = cur[a]; bool fb = true;
                    for (; s < n + 2; ++s) {
                        int y = pl[pos];
                        if (usable[y] && P[y] >= mem[a]) { fb = false; break; }
                        pos += step[a]; if (pos >= n) pos -= n;
                    }
                    const int t = fb ? n : s;
                    if (!fb && pl[(home[a] + (long)t * step[a]) % n] != x) { fprintf(stderr, "mismatch %ld\n", (long)i); return 2; }
                    int today = fb ? n + 2 - cur[a] : t - cur[a] + 1;
                    if (fb) {
                        // the engine's U: exact at the batch start, min(U, mem - 1) after a failed rank-0 walk
                        if (mem[a] <= Ueng[pool[a]]) {
                            ++eng_fb_walks; eng_fb_walk += n + 2 - cur[a];
                            if (r == 0) Ueng[pool[a]] = mem[a] - 1;
                            // the same with a capacity bound per memory value at the chunk start (rank r >= C: no walk)
                            long C = 0;
                            for (int y : pl) if (usable[y] && snaps.back()[y] >= mem[a]) C += snaps.back()[y] / mem[a];
                            if (C > r) { ++cap_fb_walks; cap_fb_walk += n + 2 - cur[a]; }
                        }
                    }
                    if (fb) {  // the engine's U bound: no usable permit count of the pool reaches mem (exact here)
                        int U = -1;
                        for (int y : pl) if (usable[y]) U = max(U, P[y]);
                        if (mem[a] > U) today = 0;
                    }
                    int help = today;
                    if (have) {
                        ++helped;
                        long key = (long)pool[a] << 32 | mem[a];
                        auto it = capm.find(key);
                        long C;
                        if (it == capm.end()) {
                            C = 0;
                            for (int y : pl) if (usable[y] && S[y] >= mem[a]) C += S[y] / mem[a];
                            capm[key] = C;
                        } else C = it->second;
                        if (C <= r || (fb && today == 0)) help = 0;  // proven fallback
                        else {
                            long cum = 0; long pp = home[a] % n; int lb = 0;
                            for (; lb < n + 2; ++lb) {
                                int y = pl[pp];
                                if (usable[y] && S[y] >= mem[a]) { cum += S[y] / mem[a]; if (cum > r) break; }
                                pp += step[a]; if (pp >= n) pp -= n;
                            }
                            const int st = max(cur[a], lb);
                            help = fb ? n + 2 - st : t - st + 1;
                            if (help < 1) { fprintf(stderr, "bound violated at %ld: t %d lb %d\n", (long)i, t, lb); return 3; }
                        }
                    }
                    if (fb) { ++fb_total; fb_proven += help == 0; fb_walk_today += today; fb_walk_help += help; }
                    steps_today += today; steps_help += help;
                    long_today += today > 16; long_help += help > 16;
                    cur[a] = fb ? n : t;
                    P[x] -= mem[a];
                } else {
                    // concurrent: apply the reference's effect
                    auto& e = cm[(long)x << 20 | slot[a]];
                    if (e.first >= 1) { e.first--; e.second++; }
                    else { P[x] -= mem[a]; e.second++; int n2 = e.first + maxc[a] - 1; e.first = (n2 % maxc[a] == 0) ? n2 - maxc[a] : n2; }
                }
            }
        }
    }
    printf("engine-like U: fallback walks %ld (%ld steps); with a chunk-start capacity bound %ld (%ld steps)\n",
           eng_fb_walks, eng_fb_walk, cap_fb_walks, cap_fb_walk);
    printf("%s cw %d lag %d: %ld mc1 decisions (%ld with a helper snapshot)\n", d.c_str(), CW, L, n1, helped);
    printf("  walk steps: today %.2f / decision, with helpers %.2f\n", (double)steps_today / n1, (double)steps_help / n1);
    printf("  walks > 16 steps: today %ld, with helpers %ld\n", long_today, long_help);
    printf("  fallbacks %ld: proven by the snapshot capacity %ld; their walk steps today %ld, with helpers %ld\n", fb_total,
           fb_proven, fb_walk_today, fb_walk_help);
}
