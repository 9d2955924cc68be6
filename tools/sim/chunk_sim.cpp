// Analysis simulator: sequential reference + chunked speculative resolution (counts passes)
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>
#include <string>
#include <unordered_map>
#include <algorithm>
using namespace std;
typedef uint64_t u64;

template <class T> vector<T> load(const string& d, const char* n) {
    string p = d + "/" + n + ".bin";
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) { perror(p.c_str()); exit(1); }
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    vector<T> v(sz / sizeof(T)); fread(v.data(), 1, sz, f); fclose(f); return v;
}
static inline u64 splitmix64(u64 x) { x += 0x9E3779B97F4A7C15ULL; x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL; x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL; return x ^ (x >> 31); }
static inline uint32_t rng_index(u64 seed, u64 seq, uint32_t n) { u64 u = splitmix64(seed ^ (seq * 0x9E3779B97F4A7C15ULL)) >> 32; return (uint32_t)((u * (u64)n) >> 32); }

struct W {
    vector<int32_t> perm, mpool, bpool, usable, home, step, mem, maxc, pool, slot, act, out; vector<int64_t> acq_off, rel_off, rel_aid; vector<uint8_t> fl; u64 seed;
    vector<int32_t> hm, hb;
};
struct CE { int c, ops; };
struct State {
    vector<int32_t> P; unordered_map<u64, CE> cm;
    u64 key(int x, int s) const { return ((u64)x << 32) | (uint32_t)s; }
};

W w; int NB;
const vector<int32_t>& poolv(int p) { return p ? w.bpool : w.mpool; }
const vector<int32_t>& hv(int p) { return p ? w.hb : w.hm; }

// feasibility of a try at x for action a
static bool feasible(State& S, int x, int a) {
    if (!w.usable[x]) return false;
    if (w.maxc[a] == 1) return S.P[x] >= w.mem[a];
    auto it = S.cm.find(S.key(x, w.slot[a]));
    int c = it == S.cm.end() ? 0 : it->second.c;
    return c >= 1 || S.P[x] >= w.mem[a];
}
static void acquire(State& S, int x, int a, bool force) {
    int m = w.mem[a], mc = w.maxc[a];
    if (mc == 1) { S.P[x] -= m; return; }
    CE& e = S.cm[S.key(x, w.slot[a])];
    if (e.c >= 1) { e.c--; e.ops++; return; }
    S.P[x] -= m;  // try succeeded (or force)
    e.ops++;
    int n2 = e.c + mc - 1;
    e.c = (n2 % mc == 0) ? n2 - mc : n2;
}
static void release(State& S, int x, int a) {
    int m = w.mem[a], mc = w.maxc[a];
    if (mc == 1) { S.P[x] += m; return; }
    auto it = S.cm.find(S.key(x, w.slot[a]));
    if (it == S.cm.end()) { fprintf(stderr, "nosuch\n"); return; }
    CE& e = it->second; e.ops--; int n2 = e.c + 1;
    if (n2 % mc == 0) { e.c = n2 - mc; S.P[x] += m; } else e.c = n2;
    if (e.ops == 0) S.cm.erase(it);
}
// true decision at current state, walking from step s0 (all earlier steps known infeasible); returns target, *fb, *sout
static int decide(State& S, int64_t i, int a, int s0, int* fb, int* sout) {
    int p = w.pool[a]; const auto& pl = poolv(p); int n = pl.size();
    long pos = (w.home[a] + (long)s0 * w.step[a]) % n;
    for (int s = s0; s < n; ++s) {
        int x = pl[pos];
        if (feasible(S, x, a)) { *fb = 0; *sout = s; return x; }
        pos += w.step[a]; if (pos >= n) pos -= n;
    }
    *fb = 1; *sout = n;
    const auto& H = hv(p);
    return H[rng_index(w.seed, (u64)i, H.size())];
}

int main(int argc, char** argv) {
    string d = argv[1]; int WCH = argc > 2 ? atoi(argv[2]) : 64; int mode = argc > 3 ? atoi(argv[3]) : 1;
    w.perm = load<int32_t>(d, "perm"); w.mpool = load<int32_t>(d, "mpool"); w.bpool = load<int32_t>(d, "bpool"); w.usable = load<int32_t>(d, "usable");
    w.home = load<int32_t>(d, "home"); w.step = load<int32_t>(d, "step"); w.mem = load<int32_t>(d, "mem"); w.maxc = load<int32_t>(d, "maxc");
    w.pool = load<int32_t>(d, "pool"); w.slot = load<int32_t>(d, "slot"); w.act = load<int32_t>(d, "act"); w.out = load<int32_t>(d, "out");
    w.acq_off = load<int64_t>(d, "acq_off"); w.rel_off = load<int64_t>(d, "rel_off"); w.rel_aid = load<int64_t>(d, "rel_aid"); w.fl = load<uint8_t>(d, "fl");
    w.seed = load<u64>(d, "seed")[0];
    for (int x : w.mpool) if (w.usable[x]) w.hm.push_back(x);
    for (int x : w.bpool) if (w.usable[x]) w.hb.push_back(x);
    NB = w.acq_off.size() - 1;
    int64_t N = w.act.size();
    // ------------------------------------------------ chunked speculative replay with exact validation
    State S; S.P = w.perm;
    vector<int32_t> out(N, -9);
    int A = w.home.size();
    vector<int> cur(A, 0);
    long passes = 0, probes = 0, wave_probe_max = 0, n_rej = 0, rej_same = 0, maxcm = 0, rej_conc = 0, rej_fb = 0;
    long waves = 0, n_stop = 0, stop_conc = 0, stop_ovf = 0, n_ext = 0, ext_gain = 0, n_resume_bad = 0;
    vector<int> spec_t(WCH), spec_s(WCH), spec_fb(WCH), spec_k(WCH);
    vector<char> kfv(WCH, 1);
    unordered_map<int, int> rankmap;
    for (int b = 0; b < NB; ++b) {
        for (int64_t r = w.rel_off[b]; r < w.rel_off[b + 1]; ++r) { int64_t aid = w.rel_aid[r]; release(S, out[aid], w.act[aid]); }
        maxcm = max(maxcm, (long)S.cm.size());
        fill(cur.begin(), cur.end(), 0);
        for (int64_t c0 = w.acq_off[b]; c0 < w.acq_off[b + 1]; c0 += WCH) {
            int64_t end = min(c0 + WCH, w.acq_off[b + 1]);
            int64_t f = c0;
            while (f < end) {
                ++passes;
                // speculation for lanes [f, end) against state at f
                rankmap.clear();
                long wmax = 0;
                for (int64_t i = f; i < end; ++i) {
                    int a = w.act[i]; int p = w.pool[a]; const auto& pl = poolv(p); int n = pl.size();
                    int r = (mode >= 1 && (w.maxc[a] == 1 || mode >= 4)) ? rankmap[a]++ : 0;
                    int s = cur[a]; long pos = (w.home[a] + (long)s * w.step[a]) % n; long cum = 0; int tg = -1, fb = 1; long pr = 0;
                    for (; s < n; ++s) {
                        int x = pl[pos]; ++pr;
                        if (w.usable[x]) {
                            long cap;
                            if (w.maxc[a] == 1) cap = S.P[x] >= 0 ? S.P[x] / w.mem[a] : 0;
                            else if (mode >= 4) { auto it = S.cm.find(S.key(x, w.slot[a])); long c = it == S.cm.end() ? 0 : it->second.c; cap = c + (S.P[x] >= 0 ? S.P[x] / w.mem[a] : 0) * w.maxc[a]; if (cum + cap > r) { long k = r - cum; spec_k[i - c0] = k < c ? -1 : (int)((k - c) % w.maxc[a]); } }
                            else cap = feasible(S, x, a) ? 1 : 0;
                            if (cum + cap > r) { tg = x; fb = 0; break; }
                            cum += cap;
                        }
                        pos += w.step[a]; if (pos >= n) pos -= n;
                    }
                    if (fb) { const auto& H = hv(p); tg = H[rng_index(w.seed, (u64)i, H.size())]; }
                    spec_t[i - c0] = tg; spec_s[i - c0] = s; spec_fb[i - c0] = fb;
                    probes += pr; wmax = max(wmax, pr);
                }
                wave_probe_max += wmax;
                int64_t lim = end;
                if (mode >= 2) {
                    // bucketed totals: lane fits if first in its bucket or bucket total <= P[t] at f
                    int B = (mode == 2 || mode == 6) ? 4096 : 1 << 20;
                    static vector<long> tot(1 << 20, 0); static vector<int64_t> firstl(1 << 20, -1);
                    vector<int> touched;
                    for (int64_t i = f; i < end; ++i) {
                        int a = w.act[i]; int t = spec_t[i - c0]; int bk = (unsigned)(t * 2654435761u) % B; if (B == (1<<20)) bk = t;
                        long cons = w.mem[a];
                        if (w.maxc[a] > 1 && mode < 4) { auto it = S.cm.find(S.key(t, w.slot[a])); int c = it == S.cm.end() ? 0 : it->second.c; cons = c >= 1 ? 0 : w.mem[a]; }
                        if (w.maxc[a] > 1 && mode >= 4) cons = spec_fb[i - c0] ? w.mem[a] : (spec_k[i - c0] == 0 ? w.mem[a] : 0);
                        if (firstl[bk] < 0) { firstl[bk] = i; touched.push_back(bk); }
                        tot[bk] += cons;
                    }
                    static vector<long> pre(1 << 20, 0);
                    bool stopped = false;
                    for (int64_t i = f; i < end; ++i) {
                        int a = w.act[i]; int t = spec_t[i - c0]; int bk = (unsigned)(t * 2654435761u) % B; if (B == (1<<20)) bk = t;
                        bool kf = firstl[bk] == i || spec_fb[i - c0] || tot[bk] <= S.P[t];
                        if (mode >= 5) {
                            // exact per-invoker prefix: the lanes before i at t leave room for i
                            long cons = w.mem[a];
                            if (w.maxc[a] > 1) cons = spec_fb[i - c0] ? w.mem[a] : (spec_k[i - c0] == 0 ? w.mem[a] : 0);
                            kf = spec_fb[i - c0] || pre[t] + cons <= S.P[t] || pre[t] == 0 && firstl[bk] == i;
                            pre[t] += cons;
                        }
                        bool ck = false;
                        if (w.maxc[a] > 1 && firstl[bk] != i && mode < 4) { if (kf) ck = true; kf = false; }
                        if (w.maxc[a] > 1 && mode >= 4) {
                            // shared key: another action with the same slot in [f,i) -> uncertain; concurrent fallback of same key earlier -> uncertain
                            for (int64_t j = f; j < i; ++j) { int aj = w.act[j]; if (w.slot[aj] == w.slot[a] && (aj != a || spec_fb[j - c0])) { if (kf) ck = true; kf = false; break; } }
                        }
                        kfv[i - c0] = kf;
                        if (!kf && !stopped) { lim = i; stopped = true; if (ck) ++stop_conc; else if (tot[bk] > S.P[t]) ++stop_ovf; if (mode < 7) break; }
                    }
                    for (int bk : touched) { tot[bk] = 0; firstl[bk] = -1; }
                    if (mode >= 5) for (int64_t i = f; i < end; ++i) pre[spec_t[i - c0]] = 0;
                }
                // exact validation in stream order
                int64_t i = f;
                bool ext_used = false;
                vector<int> ext_acts, ext_tg;
                for (; i < end; ++i) {
                    int a = w.act[i]; int fb, so;
                    int t = decide(S, i, a, cur[a], &fb, &so);
                    bool okk = (t == spec_t[i - c0]) && (fb == spec_fb[i - c0]);
                    bool aclash = false, aclash_any = false;
                    for (int q : ext_acts) if (q == a) aclash_any = true;
                    if (mode == 9) aclash = aclash_any;
                    if (mode >= 7 && i == lim && lim < end && w.maxc[a] == 1 && !ext_used && !aclash) {
                        // extension: the stop lane is re-decided exactly in this pass; later lanes known to fit that
                        // are neither of its action nor at its new target commit too
                        ext_used = mode == 7;
                        ++n_ext;
                        if (!spec_fb[i - c0]) {  // the kernel resumes the walk at the speculated step: same answer?
                            int fb2, so2;
                            const int t2 = decide(S, i, a, spec_s[i - c0], &fb2, &so2);
                            if (t2 != t || fb2 != fb) {
                                ++n_resume_bad;
                                if (n_resume_bad <= 5) fprintf(stderr, "resume mismatch at %ld: exact %d/%d from cur %d, resumed %d/%d from %d (aclash %d)\n", (long)i, t, fb, cur[a], t2, fb2, spec_s[i - c0], (int)aclash_any);
                            }
                        }
                        int64_t l2 = i + 1;
                        ext_acts.push_back(a); ext_tg.push_back(t);
                        auto clash = [&](int64_t k) {
                            for (size_t q = 0; q < ext_acts.size(); ++q)
                                if (w.act[k] == ext_acts[q] || spec_t[k - c0] == ext_tg[q]) return true;
                            return false;
                        };
                        while (l2 < end && kfv[l2 - c0] && !clash(l2)) ++l2;
                        ext_gain += l2 - i - 1;
                        lim = l2;
                        acquire(S, t, a, fb); out[i] = t;
                        if (w.maxc[a] == 1) cur[a] = fb ? (w.pool[a] ? w.bpool.size() : w.mpool.size()) : so;
                        continue;
                    }
                    if (mode >= 2 && i >= lim) { if (!okk) {} ++n_stop; acquire(S, t, a, fb); out[i] = t; if (w.maxc[a] == 1) cur[a] = fb ? (w.pool[a] ? w.bpool.size() : w.mpool.size()) : so; ++i; break; }
                    if (mode >= 2 && !okk) { fprintf(stderr, "UNSOUND at %ld\n", (long)i); exit(2); }
                    acquire(S, t, a, fb);
                    out[i] = t;
                    if (w.maxc[a] == 1) cur[a] = fb ? w.pool[a] ? w.bpool.size() : w.mpool.size() : so;
                    if (!okk) {
                        ++n_rej; if (w.maxc[a] > 1) ++rej_conc; if (fb || spec_fb[i - c0]) ++rej_fb;
                        // was an earlier lane in [f,i) of the same action?
                        for (int64_t j = f; j < i; ++j) if (w.act[j] == a) { ++rej_same; break; }
                        ++i; break;
                    }
                }
                f = i;
            }
        }
    }
    long bad = 0; for (int64_t i = 0; i < N; ++i) if (out[i] != w.out[i]) ++bad;
    printf("%s W=%d mode=%d: mismatches=%ld passes=%ld (%.3f/lane, %.2f per chunk) rej=%ld (same-action %ld, conc %ld, fb %ld) probes/lane=%.2f wavemax/pass=%.2f maxcm=%ld stops=%ld conc=%ld ovf=%ld ext=%ld ext_gain=%ld resume_bad=%ld\n",
           d.c_str(), WCH, mode, bad, passes, (double)passes / N, (double)passes / ((double)N / WCH), n_rej, rej_same, rej_conc, rej_fb, (double)probes / N,
           (double)wave_probe_max / passes, maxcm, n_stop, stop_conc, stop_ovf, n_ext, ext_gain, n_resume_bad);
}
