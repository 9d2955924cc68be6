// Analysis: sequential replay (maxConcurrent == 1 lanes) with, per decision, the walk length from the action's
// cursor and the number of usable invokers of the pool whose permits fit the decision's memory (the candidates a
// feasibility-bitmap scan would look at).  g++ -O2 -o /tmp/feas tools/sim/feas_stats.cpp && /tmp/feas /tmp/sim/c2
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <string>
#include <algorithm>
using namespace std;
typedef uint64_t u64;
template <class T> vector<T> load(const string& d, const char* n) {
    string p = d + "/" + n + ".bin";
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) { perror(p.c_str()); exit(1); }
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    vector<T> v(sz / sizeof(T)); if (fread(v.data(), 1, sz, f) != (size_t)sz) exit(1); fclose(f); return v;
}
int main(int argc, char** argv) {
    string d = argv[1];
    auto perm = load<int32_t>(d, "perm"), mpool = load<int32_t>(d, "mpool"), bpool = load<int32_t>(d, "bpool"),
         usable = load<int32_t>(d, "usable"), home = load<int32_t>(d, "home"), step = load<int32_t>(d, "step"),
         mem = load<int32_t>(d, "mem"), maxc = load<int32_t>(d, "maxc"), pool = load<int32_t>(d, "pool"),
         act = load<int32_t>(d, "act"), out = load<int32_t>(d, "out");
    auto acq_off = load<int64_t>(d, "acq_off"), rel_off = load<int64_t>(d, "rel_off"), rel_aid = load<int64_t>(d, "rel_aid");
    vector<int32_t> P = perm;
    int NB = acq_off.size() - 1, A = home.size();
    vector<int> cur(A, 0);
    // histograms: walk length buckets and feasible-count buckets, for walks > 16 steps
    long nlong = 0, n = 0, hist_f[8] = {0}, hist_w[8] = {0}, feas_le64_long = 0, sum_f_long = 0;
    auto bucket = [](long v) { return v <= 0 ? 0 : v <= 16 ? 1 : v <= 64 ? 2 : v <= 128 ? 3 : v <= 256 ? 4 : v <= 512 ? 5 : v <= 2048 ? 6 : 7; };
    for (int b = 0; b < NB; ++b) {
        for (int64_t r = rel_off[b]; r < rel_off[b + 1]; ++r) {
            int64_t aid = rel_aid[r]; int a = act[aid];
            if (maxc[a] == 1 && out[aid] >= 0) P[out[aid]] += mem[a];
        }
        fill(cur.begin(), cur.end(), 0);
        for (int64_t i = acq_off[b]; i < acq_off[b + 1]; ++i) {
            int a = act[i]; if (maxc[a] != 1) continue;
            const auto& pl = pool[a] ? bpool : mpool; int nn = pl.size();
            long pos = (home[a] + (long)cur[a] * step[a]) % nn; int s = cur[a], t = -1;
            for (; s < nn; ++s) { int x = pl[pos]; if (usable[x] && P[x] >= mem[a]) { t = x; break; } pos += step[a]; if (pos >= nn) pos -= nn; }
            int walk = s - cur[a] + 1;
            long F = 0; for (int x : pl) F += usable[x] && P[x] >= mem[a];
            ++n; ++hist_w[bucket(walk)];
            if (walk > 16) { ++nlong; ++hist_f[bucket(F)]; feas_le64_long += F <= 64; sum_f_long += F; }
            int tg = t >= 0 ? t : out[i];
            if (tg != out[i]) { fprintf(stderr, "mismatch at %ld\n", (long)i); return 2; }
            P[tg] -= mem[a];
            cur[a] = t >= 0 ? s : nn;
        }
    }
    printf("%s: %ld decisions, walks>16: %ld; feasible<=64 among them: %ld, mean feasible %.1f\n", d.c_str(), n, nlong,
           feas_le64_long, nlong ? (double)sum_f_long / nlong : 0.0);
    const char* lb[8] = {"0", "1-16", "17-64", "65-128", "129-256", "257-512", "513-2048", ">2048"};
    printf("walk length:"); for (int k = 0; k < 8; ++k) printf(" %s:%ld", lb[k], hist_w[k]); printf("\n");
    printf("feasible (long walks):"); for (int k = 0; k < 8; ++k) printf(" %s:%ld", lb[k], hist_f[k]); printf("\n");
}
