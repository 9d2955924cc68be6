// owgs_host.cpp -- host runtime behind include/owgs.h.
//
// Holds the controller-shard structure that changes rarely (invoker list, managed/blackbox split, step sizes,
// cluster size) and mirrors ShardingContainerPoolBalancerState (SCPB:449-585) line by line; everything touched per
// activation (slot permits, concurrency maps, outputs) lives in HBM and is updated by the HIP engine
// (owgs_kernels.hip).  No CPU fallback exists: without a HIP device every compute entry point fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/owgs.h"
#include "owgs_internal.h"

typedef unsigned long long u64;

extern "C" hipError_t owgs_launch_hash(const OwgsHashArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_lookup(const OwgsLookupArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_selftest(int* bad, int trials, hipStream_t s);
extern "C" hipError_t owgs_launch_prepare(const OwgsPrepArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_prepass(const OwgsPrepassArgs* a, int32_t* cstart, int64_t max_chunks,
                                          hipStream_t s);
extern "C" hipError_t owgs_launch_ovf_clear(const OwgsOvf* O, hipStream_t s);
extern "C" hipError_t owgs_launch_ovf_rehash(const uint2* old_t, int32_t old_cap, const OwgsOvf* O, int32_t* err,
                                            hipStream_t s);
extern "C" hipError_t owgs_launch_relpos(const OwgsRelposArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_relflags(const int64_t* rel_aid, int64_t n_rel, const int32_t* out_inv,
                                           uint8_t* rel_flags, hipStream_t s);
extern "C" hipError_t owgs_launch_release_seq(const OwgsReleaseArgs* a, hipStream_t s);
extern "C" size_t owgs_release_scratch_bytes(int32_t n);
extern "C" hipError_t owgs_launch_engine(const OwgsEngineArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_engine_multi(const OwgsEngineArgs* a, int k, hipStream_t s);
extern "C" hipError_t owgs_launch_engine_multi_dev(const OwgsEngineArgs* a_host, const OwgsEngineArgs* a_dev, int k,
                                                   hipStream_t s);
extern "C" int32_t owgs_coprime_max(void);
extern "C" hipError_t owgs_launch_coprime(const int32_t* xs, int32_t n_pools, int32_t* out, int32_t out_stride,
                                          int32_t* counts, hipStream_t s);
extern "C" hipError_t owgs_launch_slots(const int64_t* mem_bytes, int32_t from, int32_t n, int32_t cluster,
                                       int64_t min_bytes, int32_t* permits, hipStream_t s);
extern "C" hipError_t owgs_launch_seq(const OwgsSeqArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_seq_rehash(const uint4* old, int32_t old_cap, const OwgsSeqArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_seq_migrate(const uint32_t* ct_keys, const uint32_t* ct_vals, int32_t n_ct,
                                              const uint2* ovf, int32_t ovf_cap, const uint32_t* w_keys,
                                              const uint32_t* w_vals, int32_t w_cap, const OwgsSeqArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_seq_lookup(const OwgsSeqArgs* a, int32_t inv, int32_t slot, int32_t* out, hipStream_t s);
extern "C" hipError_t owgs_launch_usable_rows(const uint8_t* status, int64_t stride, int32_t n, int32_t rows,
                                              uint32_t* bits, int32_t n_words, hipStream_t s);
extern "C" hipError_t owgs_launch_usable(const uint8_t* status, int32_t n, uint32_t* bits, int32_t n_words,
                                        hipStream_t s);
extern "C" hipError_t owgs_launch_slot_scan(const uint32_t* ct_keys, const uint2* ovf, int32_t ovf_cap,
                                           const uint32_t* w_keys, int32_t w_cap, const int32_t* wkey, uint32_t* cand,
                                           hipStream_t s);
extern "C" hipError_t owgs_launch_ack_parse(const OwgsAckParseArgs* a, hipStream_t st);
extern "C" hipError_t owgs_launch_aid_decode(const char* aid32, int32_t n, const uint8_t* cflags, ulonglong2* key,
                                             uint8_t* info, int32_t* inst, const int32_t* inv, hipStream_t st);
extern "C" hipError_t owgs_launch_act_init(const OwgsActTable* T, hipStream_t st);
extern "C" hipError_t owgs_launch_act_rehash(const OwgsActTable* O, const OwgsActTable* T, hipStream_t st);
extern "C" hipError_t owgs_launch_act_track(const OwgsActTable* T, const ulonglong2* key, int32_t n,
                                            const int32_t* action, const int32_t* ticket, int32_t* slot,
                                            uint8_t* state, int32_t* out_ticket, uint8_t* out_existed,
                                            unsigned long long* counters, hipStream_t st);
extern "C" hipError_t owgs_launch_ack_complete(const OwgsActTable* T, const OwgsAckCompleteArgs* a, hipStream_t st);
extern "C" hipError_t owgs_launch_ack_flags(int32_t n, const uint8_t* info, const uint8_t* rflags,
                                            const uint8_t* out_kind, uint8_t* out_flags, hipStream_t st);
extern "C" hipError_t owgs_launch_health_init(uint8_t* s, uint32_t* ring, int64_t* last, int64_t* tick, int64_t* mem,
                                              int32_t* tests, int32_t from, int32_t to, hipStream_t st);
extern "C" size_t owgs_health_sort_bytes(int32_t n, int32_t bits);
extern "C" hipError_t owgs_launch_health_batch(const int32_t* ev_inv, const uint8_t* ev_kind, const int64_t* ev_t,
                                               const int64_t* ev_mem, int32_t n, int32_t bits, void* temp,
                                               size_t temp_bytes, int32_t* key_out, int32_t* idx_in,
                                               int32_t* idx_out, int64_t* packed, int32_t* seg_beg, int32_t* seg_end,
                                               int32_t* reg_first, int32_t* pad_src, uint8_t* s, uint32_t* ring,
                                               int64_t* last, int64_t* tick, int64_t* mem, int32_t* tests,
                                               int32_t old_size, int32_t new_size, int64_t now, hipStream_t st);
extern "C" size_t owgs_msg_scratch_bytes(int32_t n, int32_t n_topics, int32_t bits);
extern "C" hipError_t owgs_launch_msg_plan(const OwgsMsgArgs* a, int32_t bits, void* temp, size_t temp_bytes,
                                           uint32_t* key_sorted, int32_t* iota, int64_t* len_sorted, int32_t* cnt,
                                           hipStream_t st);
extern "C" hipError_t owgs_launch_msg_write(const OwgsMsgArgs* a, hipStream_t st);
extern "C" size_t owgs_engine_lds_bytes(int n_slots, int pool_mode, int n_ids, int nm, int nb, int n_actions);
// the narrow geometry (owgs_engine_narrow.hip): same ABI, 7 x 32-lane chunks
extern "C" size_t owgs_engine_lds_bytes_narrow(int n_slots, int pool_mode, int n_ids, int nm, int nb, int n_actions);
extern "C" hipError_t owgs_launch_prepass_narrow(const OwgsPrepassArgs* a, int32_t* cstart, int64_t max_chunks,
                                                 hipStream_t s);
extern "C" hipError_t owgs_launch_engine_narrow(const OwgsEngineArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_engine_multi_narrow(const OwgsEngineArgs* a, int k, hipStream_t s);
extern "C" hipError_t owgs_launch_engine_multi_dev_narrow(const OwgsEngineArgs* a_host, const OwgsEngineArgs* a_dev,
                                                          int k, hipStream_t s);
#define OWGS_WL_NARROW (OWGS_EW * 32)
extern "C" hipError_t owgs_launch_w_rebuild(const OwgsWRebuildArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_stage_releases(const OwgsStageArgs* a, hipStream_t s);
extern "C" hipError_t owgs_launch_relmeta(int32_t n, const int32_t* act, const int32_t* act_mem,
                                          const int32_t* act_maxc, const int32_t* act_slot, int32_t* mem,
                                          int32_t* maxc, int32_t* slot, hipStream_t s);
extern "C" hipError_t owgs_launch_w_update(const OwgsWUpdateArgs* a, hipStream_t s);
extern "C" size_t owgs_resident_image_bytes(int32_t n_slots, int32_t n_ids);
extern "C" hipError_t owgs_launch_resident(const OwgsResArgs* a, size_t lds_bytes, hipStream_t s);
extern "C" hipError_t owgs_launch_w_relgather(const int64_t* rel_aid, int32_t n, const int32_t* out_inv,
                                              const int32_t* act, const int32_t* act_mem, const int32_t* act_maxc,
                                              const int32_t* act_slot, int32_t* inv, int32_t* mem, int32_t* maxc,
                                              int32_t* slot, hipStream_t s);

namespace {

// diagnostic environment switches, read once per process (not on every call)
struct EnvOpts {
    int opts = 0, cw = 0, deal = -1, variant = -1;
    bool trace = false, feat_all = false;
    // owgs_process_batch through the resident engine: on/off, the largest call (releases + publishes) it takes, and
    // its idle time before it writes the state back and exits (OWGS_RESIDENT=0 sends every call down the chain)
    int res = 1, res_max = 1024;
    long long res_idle_us = 20000;
    // ... and its lifetime: it exits between calls once this long after its launch even when busy (it holds a hardware
    // queue that another context's stream may share; GPU_MAX_HW_QUEUES is 4), the next call relaunches it
    long long res_life_us = 100000;
    // watched pairs (after updateCluster) on the resident engine (0: such calls take the launch chain, as in round 4)
    int res_watch = 1;
    int res_eager = 1;  // OWGS_RES_EAGER=0: after a chained call the engine is relaunched by the next small call only
    // (tests) the doorbell's and the walk-cursor generation's values at the context's first launch: start a context
    // just below their wrap limits
    long long res_call_base = 0, res_gen_base = 0;
    // the resident engine's speculative walks: walk steps each publish probes on its own before the in-order
    // validation (0: every decision walked one at a time)
    int res_spec = 16;
    int res_cspec = 0;  // OWGS_RES_CSPEC: walk steps a concurrent publish speculates (0: max(4, res_spec / 4))
    int res_cspec_pre = 0;  // OWGS_RES_CSPEC_PRE: ... when the helper speculates the next chunk ahead (0: as above)
    int res_split = 1;  // OWGS_RES_SPLIT: helper waves (0-3) for the concurrent speculation; 0 = wave 0 itself
    // OWGS_RES_PRE=0: the helper wave does not speculate a run's next chunk while wave 0 decides the current one
    int res_pre = 1;
    // owgs_replay_device through the resident engine's stream mode (one wave deciding, speculative walks) instead of
    // the chunked engine, where it applies (identity pools, no watched pairs)
    int spec_replay = 0;
    EnvOpts() {
        if (const char* e = getenv("OWGS_SPEC_REPLAY")) spec_replay = atoi(e);
        if (const char* e = getenv("OWGS_RESIDENT")) res = atoi(e);
        if (const char* e = getenv("OWGS_RES_SPEC")) res_spec = atoi(e);
        if (const char* e = getenv("OWGS_RES_CSPEC")) res_cspec = atoi(e);
        if (const char* e = getenv("OWGS_RES_CSPEC_PRE")) res_cspec_pre = atoi(e);
        if (const char* e = getenv("OWGS_RES_SPLIT")) res_split = atoi(e);
        if (const char* e = getenv("OWGS_RES_PRE")) res_pre = atoi(e);
        if (const char* e = getenv("OWGS_RES_MAX")) res_max = atoi(e);
        if (const char* e = getenv("OWGS_RES_IDLE_US")) res_idle_us = atoll(e);
        if (const char* e = getenv("OWGS_RES_LIFE_US")) res_life_us = atoll(e);
        if (const char* e = getenv("OWGS_RES_WATCH")) res_watch = atoi(e);
        if (const char* e = getenv("OWGS_RES_EAGER")) res_eager = atoi(e);
        if (const char* e = getenv("OWGS_RES_CALL_BASE")) res_call_base = atoll(e);
        if (const char* e = getenv("OWGS_RES_GEN_BASE")) res_gen_base = atoll(e);
        feat_all = getenv("OWGS_FEAT_ALL") != nullptr;  // the general engine for every launch (A/B diagnostics)
        if (const char* e = getenv("OWGS_VARIANT")) variant = atoi(e);  // force an engine geometry (diagnostics)
        if (const char* o = getenv("OWGS_OPTS")) opts = atoi(o);
        if (const char* e = getenv("OWGS_CW")) cw = atoi(e);
        if (const char* e = getenv("OWGS_DEAL")) deal = atoi(e);
        trace = getenv("OWGS_TRACE_FILE") != nullptr;
    }
};
const EnvOpts& env_opts() {
    static const EnvOpts e;
    return e;
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t reserve(size_t m) {
        if (m <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t bytes = (m ? m : 1) * sizeof(T);
        hipError_t e = hipMalloc((void**)&p, bytes);
        if (e == hipSuccess) n = m ? m : 1;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

int32_t d2i(double d) {  // Scala Double.toInt
    if (d != d) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return (-2147483647 - 1);
    return (int32_t)d;
}

}  // namespace
struct owgs_ctx {
    owgs_config cfg{};
    double mf = 0, bf = 0;
    std::string err;
    hipStream_t stream = nullptr;

    // ShardingContainerPoolBalancerState mirror
    std::vector<int32_t> ids;
    std::vector<int64_t> mem;
    std::vector<uint8_t> status;
    int32_t managed = 0, blackboxes = 0;
    std::vector<int32_t> msteps, bsteps;
    int32_t cluster = 1;
    int32_t n_slots = 0;
    bool pool_override[2] = {false, false};
    std::vector<int32_t> ov_ids[2];
    std::vector<uint8_t> ov_status[2];

    // derived pools
    int32_t nm = 0, nb = 0, hm = 0, hb = 0, shortcut_ok = 3;
    int32_t pool_mode = 0, n_ids = 0;  // 0: pool position p -> id p (managed) / N - nb + p (blackbox)

    // actions
    std::vector<int32_t> a_mem, a_maxc, a_slot, a_hash;
    std::vector<uint8_t> a_bb, a_cok, a_live;
    std::vector<int32_t> free_handles;  // released action handles (owgs_release_actions), reused by registrations
    std::vector<int32_t> slot_uses, slot_maxc, slot_mem;  // per fqn@version key: live handles naming it, its limits
    std::vector<std::string> slot_name;
    std::unordered_map<std::string, int32_t> slot_ids;
    // keys no live handle names: recycled (slot id reused) once no map entry and no watched pair names them any more,
    // checked on the device when registrations run out of ids (reclaim_slots); slot_epoch counts recycled keys
    std::vector<int32_t> pending_slots, free_slots;
    int64_t slot_epoch = 0, snap_slot_epoch = 0;
    DevBuf<uint32_t> d_cand;

    // device state
    DevBuf<int32_t> d_permits, d_pool_words, d_hlist, d_act_slot, d_act_hash, d_act_mem, d_act_maxc, d_steps,
        d_cpx, d_err;
    // the primary table's entries right after the chunked engine's last rebuild of it, kept across launches (a
    // launch rebuilds once its entries grew by OWGS_CTC / 8 since then; 0 after a restore: as if never rebuilt)
    DevBuf<int32_t> d_clast;
    int32_t steps_stride = 0;  // d_steps = [managed list | blackbox list], each steps_stride entries
    DevBuf<int64_t> d_mem_bytes;  // userMemory of every invoker (updateCluster recomputes all slots from it)
    DevBuf<uint8_t> d_status;
    DevBuf<uint32_t> d_usable, d_ct_keys, d_ct_vals, d_ct_tmp;
    DevBuf<uint8_t> d_act_bb, d_act_cok;
    DevBuf<uint2> d_act_meta;
    DevBuf<u64> d_stats;
    // NestedSemaphore map overflow (keys beyond the LDS-sized primary table, owgs_internal.h OwgsOvf)
    DevBuf<uint2> d_ovf, s_ovf;
    DevBuf<uint32_t> d_ovf_rc;
    DevBuf<int32_t> d_ovf_touched, d_ovf_cnt;  // d_ovf_cnt = {entries (live + deleted), touched count}
    int32_t ovf_cap = 0;
    int64_t ovf_used_ub = 0;  // host upper bound of the overflow's entries (exact after a read-back)
    // the overflow's entry count copied back after engine launches without waiting (a ring of pinned words +
    // events): read when the bound above runs out.  A probe that has arrived replaces the bound; otherwise the host
    // waits for an OLDER probe than the newest -- the launches after it keep the GPU busy meanwhile -- instead of
    // draining the stream (a batch-by-batch replay then never idles the engine stream on this bound)
    static constexpr int OVF_PROBES = 4;
    int32_t* h_ovf_cnt = nullptr;                   // [OVF_PROBES]
    hipEvent_t ev_ovf[OVF_PROBES] = {};
    bool ovf_probe[OVF_PROBES] = {};                // slot recorded and not yet consumed
    int64_t ovf_probe_added[OVF_PROBES] = {};       // ovf_added at the slot's recording (its launch included)
    int64_t ovf_added = 0;                          // activations ever added to the bound
    int ovf_probe_next = 0;
    // owgs_update_health_device on identity pools: the status bytes and usable bitmap are updated on the device only;
    // the host mirror (status, healthy counts) is downloaded when a host path needs it (ev_status: the copy)
    bool status_stale = false;
    hipEvent_t ev_status = nullptr;
    // calls on one context are ordered as issued, whatever stream each names: ev_tail marks the end of the last
    // asynchronous call's work (on tail_stream); later work on another stream waits for it (order_on / tail_mark)
    hipEvent_t ev_tail = nullptr;
    hipStream_t tail_stream = nullptr;
    bool tail_valid = false;
    int32_t s_ovf_cnt = 0;    // snapshot: overflow entries (0: the snapshot had none)
    int32_t s_ovf_cap = 0;
    DevBuf<uint32_t> d_margs;  // owgs_replay_device_multi: shard argument blocks beyond the kernarg segment
    void* h_margs = nullptr;   // pinned staging of d_margs (hipHostMalloc), h_margs_bytes long
    size_t h_margs_bytes = 0;
    hipEvent_t ev_margs = nullptr;  // recorded after the last engine launch that reads d_margs / h_margs
    bool ev_margs_valid = false;
    // per-call scratch
    DevBuf<int64_t> d_off;
    DevBuf<int32_t> d_a, d_b, d_c, d_d, d_out, d_cstart, d_relx, d_relcnt, d_xslot;
    DevBuf<uint8_t> d_flags, d_rflags;
    DevBuf<u64> d_seq;
    DevBuf<int64_t> d_rel;
    DevBuf<uint4> d_rec;
    DevBuf<uint32_t> d_lix;
    DevBuf<uint32_t> d_gcur;  // per-action walk cursors (tagged by batch)
    DevBuf<unsigned long long> d_trace;  // barrier timeline (diagnostic builds, env OWGS_TRACE_FILE)
    int32_t cur_tag = 0;      // tags used so far (wraps with a clear of d_gcur)
    DevBuf<uint2> d_rel_rec, d_xmeta;
    // activationSlots (owgs_acks.hip)
    DevBuf<unsigned long long> t_tw;
    DevBuf<ulonglong2> t_tk;
    DevBuf<int2> t_tv;
    DevBuf<int32_t> t_owner;
    long long t_cap = 0, t_used = 0, t_live = 0;
    long long health_ms = 0;
    DevBuf<ulonglong2> k_key;
    DevBuf<uint8_t> k_info, k_state, k_kind, k_oflags, k_bytes, k_cfl;
    DevBuf<int32_t> k_inst, k_slot, k_tick, k_r0, k_r1, k_r2, k_r3, k_act;
    DevBuf<int64_t> k_off;
    DevBuf<char> k_aid;
    DevBuf<unsigned long long> k_cnt;
    // invoker health supervision (owgs_health.hip): persistent SoA by invoker id + per-batch scratch
    DevBuf<uint8_t> h_st, he_kind, he_temp;
    DevBuf<uint32_t> h_ring;
    DevBuf<int64_t> h_last, h_tick, h_mem, he_t, he_mem, he_packed;
    DevBuf<int32_t> h_tests, he_inv, he_key, he_idx0, he_idx1, he_beg, he_end, he_reg, he_pad;
    int32_t h_cap = 0, h_size = 0;
    hipEvent_t ev_engine[2] = {nullptr, nullptr};  // around the last owgs_engine_kernel launch
    DevBuf<unsigned long long> r_bound;  // release front end scratch (owgs_launch_release_seq)
    DevBuf<int32_t> r_idx, r_cnt, r_cval, r_cval_s, r_cbeg;
    DevBuf<uint32_t> r_ckey, r_ckey_s;
    DevBuf<uint8_t> r_sel, r_temp;
    bool ev_engine_valid = false;
    // ActivationMessage templates + serialisation scratch (owgs_msgs.hip)
    std::vector<char> ta, tb;
    std::vector<int64_t> ta_off{0}, tb_off{0};
    std::string rci = "{\"asString\":\"0\"}";  // ControllerInstanceId("0"), jsonFormat1 (InstanceId.scala:40, 59)
    bool tmpl_dirty = true;
    DevBuf<char> m_ta, m_tb, m_rci, m_tid, m_content, m_trace, m_out;
    DevBuf<int64_t> m_ta_off, m_tb_off, m_tid_off, m_tid_start, m_content_off, m_trace_off, m_len, m_len_sorted,
        m_out_off;
    DevBuf<int32_t> m_inv, m_tmpl, m_bad, m_order, m_iota, m_cnt, m_topic;
    DevBuf<uint32_t> m_key, m_key_sorted;
    DevBuf<ulonglong2> m_aid, m_cause;
    DevBuf<uint8_t> m_flags, m_temp;
    int64_t h_now = INT64_MIN;
    // watched (invoker, fqn) pairs after a slot-state reset (owgs_watch.hip; w_cap == 0: none)
    DevBuf<uint32_t> w_keys, w_vals;
    DevBuf<int32_t> w_cnt, w_wkey, w_D, w_L, w_Lcnt, w_rel;
    DevBuf<uint4> w_L2;
    DevBuf<int64_t> w_off;
    // owgs_replay_device_group: its batch offsets, the usable bitmap of each batch's health, and (during the call) the
    // first activation of the group (releases of earlier ones get their records from those decisions)
    DevBuf<int64_t> g_off;
    // large-state engine (owgs_seq.hip): a state beyond every on-chip geometry (owgs_limits) or maxConcurrent beyond
    // OWGS_MAX_CONC runs there -- permits in HBM, the NestedSemaphore maps in one HBM table q_map
    bool large = false, big_conc = false;
    DevBuf<uint4> q_map;
    int32_t q_cap = 0;
    DevBuf<int32_t> q_filled, q_state, q_look;
    DevBuf<uint4> q_cur;   // walk cursors of the large-state engine, per action {generation, step, position, 0}
    uint32_t q_gen = 1;    // the next call's first generation: cursors never outlive the call that wrote them
    int64_t q_spec = 0, q_alone = 0;  // its decisions: kept from the group speculation / decided alone
    uint64_t q_cyc[4] = {0, 0, 0, 0};  // its cycles: releases, group speculation, kept decisions, decided alone
    DevBuf<uint32_t> d_hwords;
    const uint32_t* grp_hwords = nullptr;
    int32_t grp_hstride = 0;
    int64_t grp_a0 = 0;
    DevBuf<uint8_t> w_rfl;
    int32_t w_cap = 0, w_live = 0;
    int32_t stats_par = 0, stats_last = 0;  // d_stats holds two counter blocks: the next launch's, the last one's
    int32_t cw_cache = 0;  // chunk width of the current state and actions (0: recompute)
    bool any_conc = false;  // some registered action has maxConcurrent > 1 (the engine needs its map code)
    int32_t variant = 0;   // engine geometry: 0 wide chunks, 1 narrow (large pools, owgs_engine_narrow.hip)
    // owgs_process_batch: pinned staging (inputs, outputs) and their device copies
    void* h_pin = nullptr;
    size_t h_pin_bytes = 0;
    void* h_pout = nullptr;
    size_t h_pout_bytes = 0;
    DevBuf<uint8_t> d_pin, d_pout;
    DevBuf<int32_t> f_src, f_cnt, f_tile;
    DevBuf<uint2> f_rec;
    // owgs_process_batch through the resident engine (owgs_resident.hip): its stream, the pinned control block and
    // call buffers, the call counter (the doorbell), whether a launch is live, and counters for owgs_resident_stats
    hipStream_t res_stream = nullptr;
    hipEvent_t ev_res = nullptr;
    int32_t* res_ctl = nullptr;
    int32_t* res_in = nullptr;
    char* res_out = nullptr;
    size_t res_in_cap = 0, res_out_cap = 0;
    int32_t res_call = 0;
    bool res_alive = false;
    bool res_last_served = false;  // the previous owgs_process_batch call was served by the resident engine
    int32_t res_stage = 0;
    int64_t res_n_calls = 0, res_n_launches = 0, res_n_bails = 0, res_n_chained = 0, res_n_life = 0;
    int64_t res_n_watch_calls = 0;  // served calls while watched pairs existed
    int64_t res_prof[OWGS_RES_NPROF] = {};
    int64_t res_used_max = 0, res_tombs_max = 0;  // the primary table's fill after served calls (largest seen)
    int64_t res_host_ns[2] = {};    // served calls: host time building the call (records, ranks), bell-to-answer wait
    DevBuf<uint4> d_w_sidx;         // resident engine: watched pairs by fqn@version key (built at its launch)
    DevBuf<uint2> d_w_list;
    int32_t w_scap = 0;
    uint64_t res_cache_epoch = 1, res_cache_seen = 0;  // res_meta / the watched-pair index are current when equal
    DevBuf<uint2> d_res_cur;        // per action: {cursor generation, first walk step that may fit}
    std::vector<uint2> res_meta;    // act_meta as of the live launch (every change of it stops the engine first)
    uint32_t res_gen_seen = 0;      // the last cursor generation the engine reported
    int64_t last_call_ns = 0;       // duration of the last publish / release / process_batch call, timed inside the library
    DevBuf<unsigned long long> d_spec_stats;  // stream-mode replays: summed resident-engine counters (owgs_resident_stats)
    DevBuf<uint32_t> d_claim;       // stream-mode replays: released activations (a second release is a malformed stream)
    bool spec_last = false;         // the last replay ran in stream mode
    DevBuf<unsigned long long> f_bound;  // per slot: what a fused call's releases can return (zero between calls)
    DevBuf<uint32_t> s_w_keys, s_w_vals;
    DevBuf<int32_t> s_w_wkey;
    int32_t s_w_cap = 0, s_w_live = 0;
    // snapshot
    DevBuf<int32_t> s_permits;
    DevBuf<uint32_t> s_ct_keys, s_ct_vals;
    bool has_snap = false;
    int32_t snap_slots = 0;

    int fail(int code, const char* what, hipError_t e = hipSuccess) {
        err = what;
        if (e != hipSuccess) {
            err += ": ";
            err += hipGetErrorString(e);
        }
        return code;
    }
};

#define HIPCHK(ctx, call)                                                     \
    do {                                                                      \
        hipError_t _e = (call);                                               \
        if (_e != hipSuccess) return (ctx)->fail(OWGS_EDEVICE, #call, _e);    \
    } while (0)

template <class T>
static hipError_t upload(DevBuf<T>& d, const T* h, size_t n, hipStream_t s) {
    hipError_t e = d.reserve(n);
    if (e != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    return hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, s);
}

// managed = take(managed), blackbox = takeRight(blackboxes) (SCPB:522-523) -> pool words / usable bitmap, healthy
// lists.  InvokerPool pads the health list so that position i holds invoker id i (InvokerSupervision.scala:191-207):
// then pool position p is id p (managed) or N - blackboxes + p (blackbox) and the engine keeps only a usable bitmap.
// the host mirror of the status bytes after owgs_update_health_device's device-only path
static int sync_status(owgs_ctx* c) {
    if (!c->status_stale) return OWGS_OK;
    HIPCHK(c, hipEventSynchronize(c->ev_status));
    if (!c->status.empty())
        HIPCHK(c, hipMemcpy(c->status.data(), c->d_status.p, c->status.size(), hipMemcpyDeviceToHost));
    c->status_stale = false;
    return OWGS_OK;
}

// make stream s wait for the work of the last asynchronous call when that ran on another stream (the caller may
// free or reuse nothing of ours meanwhile: every buffer an earlier call reads belongs to the context or stays the
// caller's until its stream reaches it, include/owgs.h)
static int order_on(owgs_ctx* c, hipStream_t s) {
    if (c->tail_valid && c->tail_stream != s) HIPCHK(c, hipStreamWaitEvent(s, c->ev_tail, 0));
    return OWGS_OK;
}
// the work this asynchronous call enqueued on s is the context's new tail
static int tail_mark(owgs_ctx* c, hipStream_t s) {
    if (!c->ev_tail) HIPCHK(c, hipEventCreateWithFlags(&c->ev_tail, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ev_tail, s));
    c->tail_stream = s;
    c->tail_valid = true;
    return OWGS_OK;
}

static int rebuild_pools(owgs_ctx* c) {
    int rs = sync_status(c);
    if (rs) return rs;
    c->cw_cache = 0;
    std::vector<int32_t> words, hl;
    int32_t cnt[2], hcnt[2];
    c->shortcut_ok = 3;
    const int32_t N = (int32_t)c->ids.size();
    bool identity = !c->pool_override[0] && !c->pool_override[1] && N <= c->n_slots;
    for (int32_t i = 0; identity && i < N; ++i) identity = c->ids[i] == i;
    for (int p = 0; p < 2; ++p) {
        const int32_t* pid;
        const uint8_t* pst;
        int32_t n;
        if (c->pool_override[p]) {
            pid = c->ov_ids[p].data();
            pst = c->ov_status[p].data();
            n = (int32_t)c->ov_ids[p].size();
        } else {
            const int32_t k = p == 0 ? std::min(c->managed, N) : std::min(c->blackboxes, N);
            const int32_t base = p == 0 ? 0 : N - k;
            pid = c->ids.data() + base;
            pst = c->status.data() + base;
            n = k;
        }
        cnt[p] = n;
        hcnt[p] = 0;
        for (int32_t i = 0; i < n; ++i) {
            int32_t w = OWGS_PW_UNUSABLE;
            if (pst[i] == OWGS_HEALTHY) {
                w = (pid[i] >= 0 && pid[i] < c->n_slots) ? pid[i] : OWGS_PW_BADID;
                if (w == OWGS_PW_BADID) c->shortcut_ok &= ~(1 << p);
                hl.push_back(pid[i]);
                hcnt[p]++;
            }
            words.push_back(w);
        }
    }
    c->nm = cnt[0];
    c->nb = cnt[1];
    c->hm = hcnt[0];
    c->hb = hcnt[1];
    c->pool_mode = identity ? 0 : 1;
    c->n_ids = N;
    // usable bitmap built on the device from the status bytes (d_status mirrors c->status)
    const int32_t n_words = (N + 31) / 32 + 1;
    HIPCHK(c, c->d_usable.reserve((size_t)n_words));
    HIPCHK(c, c->d_status.reserve((size_t)N));
    HIPCHK(c, owgs_launch_usable(c->d_status.p, N, c->d_usable.p, n_words, c->stream));
    HIPCHK(c, upload(c->d_pool_words, words.data(), words.size(), c->stream));
    HIPCHK(c, upload(c->d_hlist, hl.data(), hl.size(), c->stream));
    return OWGS_OK;
}

static int prepare_actions(owgs_ctx* c) {
    ++c->res_cache_epoch;  // (the resident engine's host copies of the action meta / watched-pair index)
    const int32_t n = (int32_t)c->a_mem.size();
    if (n == 0) return OWGS_OK;
    if (!c->d_steps.p) HIPCHK(c, c->d_steps.reserve(2));
    HIPCHK(c, c->d_act_meta.reserve(n));
    OwgsPrepArgs a{};
    a.hash = c->d_act_hash.p;
    a.mem = c->d_act_mem.p;
    a.maxc = c->d_act_maxc.p;
    a.bb = c->d_act_bb.p;
    a.cursor_ok = c->d_act_cok.p;
    a.n = n;
    a.nm = c->nm;
    a.nb = c->nb;
    a.msteps = c->d_steps.p;
    a.n_msteps = (int32_t)c->msteps.size();
    a.bsteps = c->d_steps.p + c->steps_stride;
    a.n_bsteps = (int32_t)c->bsteps.size();
    a.act_meta = c->d_act_meta.p;
    HIPCHK(c, owgs_launch_prepare(&a, c->stream));
    return OWGS_OK;
}

// Engine geometry for a state: 0 = wide chunks (7 x 56 lanes), 1 = narrow (7 x 32, owgs_engine_narrow.hip) when the
// wide LDS image does not fit, -1 = neither fits.  Inputs: what the state's slot image would be.
static int engine_variant(int32_t n_slots, int32_t pool_mode, int32_t n_ids, int32_t nm, int32_t nb) {
    if (n_slots > OWGS_MAX_SLOTS_CT || nm > (int32_t)OWGS_AM_POS_MASK || nb > (int32_t)OWGS_AM_POS_MASK) return -1;
    if (owgs_engine_lds_bytes(n_slots, pool_mode, n_ids, nm, nb, 0) <= OWGS_LDS_BYTES) return 0;
    if (owgs_engine_lds_bytes_narrow(n_slots, pool_mode, n_ids, nm, nb, 0) <= OWGS_LDS_BYTES) return 1;
    return -1;
}

static int lds_check(owgs_ctx* c) {
    if (c->n_slots > OWGS_MAX_SLOTS_CT) return c->fail(OWGS_ERANGE, "invoker ids beyond the concurrency-map key range");
    if (c->nm > (int32_t)OWGS_AM_POS_MASK || c->nb > (int32_t)OWGS_AM_POS_MASK)
        return c->fail(OWGS_ERANGE, "pool larger than 32767 positions");
    const int v = engine_variant(c->n_slots, c->pool_mode, c->n_ids, c->nm, c->nb);
    if (v < 0) return c->fail(OWGS_ERANGE, "slot + pool state exceeds the engine's on-chip (LDS) capacity");
    c->variant = (env_opts().variant == 1 || (env_opts().variant == 0 && v == 0)) ? env_opts().variant : v;
    return OWGS_OK;
}

static int32_t variant_wl(const owgs_ctx* c) { return c->variant ? OWGS_WL_NARROW : OWGS_WL; }

static hipError_t launch_engine(const owgs_ctx* c, const OwgsEngineArgs* A, hipStream_t s) {
    return c->variant ? owgs_launch_engine_narrow(A, s) : owgs_launch_engine(A, s);
}

static OwgsOvf ovf_args(const owgs_ctx* c) {
    OwgsOvf O{};
    O.t = c->d_ovf.p;
    O.cap = c->ovf_cap;
    O.cnt = c->d_ovf_cnt.p;
    O.rc = c->d_ovf_rc.p;
    O.touched = c->d_ovf_touched.p;
    O.n_touched = c->d_ovf_cnt.p ? c->d_ovf_cnt.p + 1 : nullptr;
    return O;
}

// The overflow holds every key the primary cannot: at most the entries it has plus one per activation of the call
// (an activation creates at most one (invoker, fqn) entry).  Keep it at least twice that (load <= 1/2); grow (and
// rehash) when the bound says so -- after reading the exact entry count back once.
// n more activations may add overflow entries: the bound grows, and so does what an outstanding count probe misses
static void ovf_add(owgs_ctx* c, int64_t n) {
    c->ovf_used_ub += n;
    c->ovf_added += n;
}
static void ovf_probes_clear(owgs_ctx* c) {
    for (int k = 0; k < owgs_ctx::OVF_PROBES; ++k) c->ovf_probe[k] = false;
}
// overflow entry-count probes: the next probe slot, or -1 while its last probe is still in flight (this launch then records none)
static int ovf_probe_slot(owgs_ctx* c, int* k_out) {
    *k_out = -1;
    if (!c->h_ovf_cnt) {
        HIPCHK(c, hipHostMalloc((void**)&c->h_ovf_cnt, owgs_ctx::OVF_PROBES * sizeof(int32_t), hipHostMallocDefault));
        for (int k = 0; k < owgs_ctx::OVF_PROBES; ++k)
            HIPCHK(c, hipEventCreateWithFlags(&c->ev_ovf[k], hipEventDisableTiming));
    }
    const int k = c->ovf_probe_next;
    if (c->ovf_probe[k] && hipEventQuery(c->ev_ovf[k]) != hipSuccess) return OWGS_OK;  // (still in flight: skip)
    *k_out = k;
    return OWGS_OK;
}
// slot k's value lands behind the work queued on s so far (the engine launch before it stores it there)
static int ovf_probe_mark(owgs_ctx* c, int k, hipStream_t s) {
    HIPCHK(c, hipEventRecord(c->ev_ovf[k], s));
    c->ovf_probe[k] = true;
    c->ovf_probe_added[k] = c->ovf_added;
    c->ovf_probe_next = (k + 1) % owgs_ctx::OVF_PROBES;
    return OWGS_OK;
}
// the bound from the newest probe that has arrived (wait_older: first wait for the second-newest outstanding one)
static int ovf_probe_refresh(owgs_ctx* c, bool wait_older) {
    int newest = -1, second = -1;
    for (int k = 0; k < owgs_ctx::OVF_PROBES; ++k) {
        if (!c->ovf_probe[k]) continue;
        if (newest < 0 || c->ovf_probe_added[k] > c->ovf_probe_added[newest]) {
            second = newest;
            newest = k;
        } else if (second < 0 || c->ovf_probe_added[k] > c->ovf_probe_added[second]) {
            second = k;
        }
    }
    if (wait_older) {
        const int w = second >= 0 ? second : newest;
        if (w < 0) return OWGS_OK;
        HIPCHK(c, hipEventSynchronize(c->ev_ovf[w]));
    }
    int best = -1;
    for (int k = 0; k < owgs_ctx::OVF_PROBES; ++k)
        if (c->ovf_probe[k] && hipEventQuery(c->ev_ovf[k]) == hipSuccess &&
            (best < 0 || c->ovf_probe_added[k] > c->ovf_probe_added[best]))
            best = k;
    if (best < 0) return OWGS_OK;
    c->ovf_used_ub = std::min(c->ovf_used_ub, (int64_t)c->h_ovf_cnt[best] + (c->ovf_added - c->ovf_probe_added[best]));
    for (int k = 0; k < owgs_ctx::OVF_PROBES; ++k)  // this probe and older ones are consumed
        if (c->ovf_probe[k] && c->ovf_probe_added[k] <= c->ovf_probe_added[best]) c->ovf_probe[k] = false;
    return OWGS_OK;
}

// overflow capacity for `used` entries plus n_new activations
static int64_t ovf_need(int64_t used, int64_t n_new) {
    // (at least 2^19 entries, 12 MB with its scratch: the per-launch bound then runs out only every ~250k
    // activations, so a batch-by-batch replay seldom has to read the count back)
    int64_t want = 2 * (used + n_new + OWGS_CTC), cap = (int64_t)1 << 19;
    while (cap < want && cap < ((int64_t)1 << 30)) cap <<= 1;
    return cap;
}

static int ensure_ovf(owgs_ctx* c, int64_t n_new, hipStream_t s) {
    auto need = [&](int64_t used) { return ovf_need(used, n_new); };
    if (c->ovf_cap >= need(c->ovf_used_ub)) return OWGS_OK;
    {  // a count that arrived meanwhile, else one of an older launch (the GPU keeps the later ones)
        int rc = ovf_probe_refresh(c, false);
        if (!rc && c->ovf_cap < need(c->ovf_used_ub)) rc = ovf_probe_refresh(c, true);
        if (rc) return rc;
        if (c->ovf_cap >= need(c->ovf_used_ub)) return OWGS_OK;
    }
    ovf_probes_clear(c);
    if (c->ovf_cap > 0) {  // exact entry count
        int32_t cnt = 0;
        HIPCHK(c, hipStreamSynchronize(s));
        HIPCHK(c, hipMemcpy(&cnt, c->d_ovf_cnt.p, sizeof(cnt), hipMemcpyDeviceToHost));
        c->ovf_used_ub = cnt;
        if (c->ovf_cap >= need(cnt)) return OWGS_OK;
    }
    const int64_t cap = need(c->ovf_used_ub);
    if (cap > ((int64_t)1 << 26)) return c->fail(OWGS_ENOMEM, "concurrency map overflow beyond 2^26 entries");
    DevBuf<uint2> nt;
    HIPCHK(c, nt.reserve((size_t)cap));
    HIPCHK(c, hipMemsetAsync(nt.p, 0, (size_t)cap * sizeof(uint2), s));
    HIPCHK(c, c->d_ovf_cnt.reserve(2));
    if (c->ovf_cap == 0) HIPCHK(c, hipMemsetAsync(c->d_ovf_cnt.p, 0, 2 * sizeof(int32_t), s));
    HIPCHK(c, c->d_ovf_rc.reserve((size_t)cap));
    HIPCHK(c, hipMemsetAsync(c->d_ovf_rc.p, 0, (size_t)cap * sizeof(uint32_t), s));
    HIPCHK(c, c->d_ovf_touched.reserve((size_t)cap));
    HIPCHK(c, c->d_ct_tmp.reserve((size_t)2 * (OWGS_CTC + cap)));
    if (c->ovf_cap > 0 && c->ovf_used_ub > 0) {  // live entries move to the larger table
        OwgsOvf O = ovf_args(c);
        O.t = nt.p;
        O.cap = (int32_t)cap;
        HIPCHK(c, hipMemsetAsync(c->d_ovf_cnt.p, 0, sizeof(int32_t), s));
        HIPCHK(c, owgs_launch_ovf_rehash(c->d_ovf.p, c->ovf_cap, &O, c->d_err.p, s));
    }
    HIPCHK(c, hipStreamSynchronize(s));
    c->d_ovf.release();
    c->d_ovf = nt;
    nt.p = nullptr;
    c->ovf_cap = (int32_t)cap;
    return OWGS_OK;
}

static int reset_ctab(owgs_ctx* c) {
    HIPCHK(c, hipMemsetAsync(c->d_ct_keys.p, 0, OWGS_CTC * sizeof(uint32_t), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_ct_vals.p, 0, OWGS_CTC * sizeof(uint32_t), c->stream));
    if (c->ovf_cap > 0) {
        const OwgsOvf O = ovf_args(c);
        HIPCHK(c, owgs_launch_ovf_clear(&O, c->stream));
    }
    c->ovf_used_ub = 0;
    ovf_probes_clear(c);
    return OWGS_OK;
}

// ---------------------------------------------------------------------------------------------- watched pairs
static OwgsWatch watch_args(const owgs_ctx* c) {
    OwgsWatch w{};
    if (c->w_cap > 0) {
        w.keys = c->w_keys.p;
        w.vals = c->w_vals.p;
        w.cap = c->w_cap;
        w.cnt = c->w_cnt.p;
        w.wkey = c->w_wkey.p;
    }
    return w;
}

static void w_drop(owgs_ctx* c) {
    ++c->res_cache_epoch;  // (the resident engine's host copies of the action meta / watched-pair index)
    c->w_keys.release();
    c->w_vals.release();
    c->w_wkey.release();
    c->w_cap = 0;
    c->w_live = 0;
}

// after a call that may have taken pairs out of W (a release that threw NoSuchElement): its live count
static int w_refresh(owgs_ctx* c, hipStream_t s) {
    if (c->w_cap <= 0) return OWGS_OK;
    int32_t live = 0;
    HIPCHK(c, hipMemcpyAsync(&live, c->w_cnt.p, sizeof(live), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->w_live = live;
    if (live <= 0) w_drop(c);
    return OWGS_OK;
}

// A reset (updateCluster SCPB:561-584, the _invokerSlots test seam) is about to discard the concurrency map: every
// pair with activations in flight (operationCount of its entry + d of the pair) becomes watched (owgs_watch.hip).
static int w_rebuild(owgs_ctx* c) {
    ++c->res_cache_epoch;  // (the resident engine's host copies of the action meta / watched-pair index)
    hipStream_t s = c->stream;
    int32_t ovf_n = 0;
    HIPCHK(c, hipStreamSynchronize(s));
    if (c->ovf_cap > 0) HIPCHK(c, hipMemcpy(&ovf_n, c->d_ovf_cnt.p, sizeof(ovf_n), hipMemcpyDeviceToHost));
    const int64_t cand = (int64_t)OWGS_CTC + ovf_n + c->w_live;
    int64_t cap = 1024;
    while (cap < 2 * cand) cap <<= 1;
    DevBuf<uint32_t> nk, nv;
    HIPCHK(c, nk.reserve((size_t)cap));
    HIPCHK(c, nv.reserve((size_t)cap));
    HIPCHK(c, c->w_cnt.reserve(1));
    HIPCHK(c, hipMemsetAsync(nk.p, 0, (size_t)cap * 4, s));
    HIPCHK(c, hipMemsetAsync(nv.p, 0, (size_t)cap * 4, s));
    HIPCHK(c, hipMemsetAsync(c->w_cnt.p, 0, 4, s));
    DevBuf<int32_t> nw;  // per-key counts of the new W
    HIPCHK(c, nw.reserve((size_t)OWGS_MAX_SLOTKEYS + 1));
    HIPCHK(c, hipMemsetAsync(nw.p, 0, ((size_t)OWGS_MAX_SLOTKEYS + 1) * 4, s));
    OwgsWRebuildArgs a{};
    a.ct_keys = c->d_ct_keys.p;
    a.ct_vals = c->d_ct_vals.p;
    a.ovf = ovf_args(c);
    if (ovf_n <= 0) a.ovf.cap = 0;
    a.old_w = watch_args(c);
    a.new_w.keys = nk.p;
    a.new_w.vals = nv.p;
    a.new_w.cap = (int32_t)cap;
    a.new_w.cnt = c->w_cnt.p;
    a.new_w.wkey = nw.p;
    HIPCHK(c, owgs_launch_w_rebuild(&a, s));
    int32_t live = 0;
    HIPCHK(c, hipMemcpyAsync(&live, c->w_cnt.p, sizeof(live), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    w_drop(c);
    if (live > 0) {
        c->w_keys = nk;
        c->w_vals = nv;
        c->w_wkey = nw;
        nk.p = nv.p = nullptr;
        nw.p = nullptr;
        c->w_cap = (int32_t)cap;
        c->w_live = live;
    } else {
        nk.release();
        nv.release();
        nw.release();
    }
    return OWGS_OK;
}

static void base_args(owgs_ctx* c, OwgsEngineArgs& A) {
    memset(&A, 0, sizeof(A));
    A.permits = c->d_permits.p;
    A.n_slots = c->n_slots;
    A.pool_mode = c->pool_mode;
    A.usable = c->d_usable.p;
    A.n_ids = c->n_ids;
    A.pool_words = c->d_pool_words.p;
    A.nm = c->nm;
    A.nb = c->nb;
    A.hlist = c->d_hlist.p;
    A.hm = c->hm;
    A.hb = c->hb;
    A.shortcut_ok = c->shortcut_ok;
    A.ct_keys = c->d_ct_keys.p;
    A.ct_vals = c->d_ct_vals.p;
    A.ct_tmp = c->d_ct_tmp.p;
    A.ct_clast = c->d_clast.p;
    A.ovf = ovf_args(c);
    A.n_actions = (int32_t)c->a_mem.size();
    A.rng_seed = c->cfg.rng_seed;
    A.stats = c->d_stats.p;
    A.err = c->d_err.p;
    A.opts = env_opts().opts;
    A.hwords = c->grp_hwords;
    A.hstride = c->grp_hstride;
    A.trace = nullptr;
    if (env_opts().trace) {  // diagnostic: a -DOWGS_TRACE engine logs its barrier timeline here
        const size_t n = (size_t)(OWGS_EW + 1) * 16384 * 2;
        if (c->d_trace.reserve(n) == hipSuccess && hipMemset(c->d_trace.p, 0, n * 8) == hipSuccess) A.trace = c->d_trace.p;
    }
}

// Chunk width of a replay.  Wide chunks amortise a pass over more activations, but lanes of different actions that
// meet at an invoker without room for both stop the pass (or cost a re-decision inside it).  How often that happens follows the capacity units the
// managed pool offers (slot MB x invokers / mean action MB): with few units (small pools, or slots split over many
// controllers) a narrow chunk wins (measured, round 2: C5 shard of 8, 23k units: 244 ms at 128 lanes vs 349 at 336;
// configs[1], 19k units: 129 vs 139 ms at 256; headline, 187k units: 34 ms at 336 vs 37 at 256).  Env OWGS_CW
// overrides (diagnostics).
#ifndef OWGS_WIDE_UNITS
#define OWGS_WIDE_UNITS 60000.0
#endif
static int32_t chunk_width(owgs_ctx* c) {
    if (c->cw_cache > 0) return c->cw_cache;  // recomputed after a state or action change (cw_cache = 0)
    double slot_mb = 0, act_mb = 0;
    const int32_t nm = std::min<int32_t>(c->nm, (int32_t)c->mem.size());
    for (int32_t i = 0; i < nm; ++i)
        slot_mb += (double)std::max<int64_t>(c->cfg.min_memory_bytes, c->mem[i] / std::max(c->cluster, 1)) / 1048576.0;
    int64_t live = 0;
    for (size_t a = 0; a < c->a_mem.size(); ++a)
        if (c->a_live[a]) {
            act_mb += c->a_mem[a];
            ++live;
        }
    const double units = live == 0 || act_mb <= 0 ? 1e9 : slot_mb / (act_mb / (double)live);
    // (with in-pass re-decisions, round 2: configs[1] 19k units 116 ms at 192 vs 119 at 128; configs[3] 221 vs 232;
    // C5 shard of 8 165 vs 173; C5 shard of 4, 34k units: 102 ms at 256 vs 106 at 192 and 117 at 128)
    int32_t cw = units >= OWGS_WIDE_UNITS ? OWGS_WL : std::min(units >= OWGS_WIDE_UNITS / 2 ? 256 : 192, OWGS_WL);
    const int v = env_opts().cw;
    if (v >= 64 && v <= OWGS_WL) cw = v;
    c->cw_cache = cw;
    return cw;
}

// chunk records of n_act activations (act != null: registered actions; else explicit per-activation walks)
static int run_prepass(owgs_ctx* c, OwgsEngineArgs& A, int32_t n_batches, const int64_t* acq_off, const int32_t* act,
                       int64_t n_act, hipStream_t s) {
    HIPCHK(c, c->d_rec.reserve((size_t)std::max<int64_t>(n_act, 1)));
    HIPCHK(c, c->d_cstart.reserve((size_t)n_batches + 1));
    int rv = lds_check(c);  // the engine geometry decides the chunk width and the record layout
    if (rv) return rv;
    const int32_t wl = variant_wl(c);
    OwgsPrepassArgs p{};
    p.n_batches = n_batches;
    p.acq_off = acq_off;
    p.act = act;
    p.act_meta = c->d_act_meta.p;
    p.act_slot = c->d_act_slot.p;
    p.xmeta = c->d_xmeta.p;
    p.xslot = c->d_xslot.p;
    const int32_t cw = std::min(chunk_width(c), wl);
    const int64_t max_chunks = n_act / cw + n_batches;
    p.cw = cw;
    A.cw = cw;
    p.geom = A.geom = OWGS_GEOM_TAG(wl);  // the geometry d_lix and the records below are sized for
    // lane dealing: concurrent lanes packed into the back waves for large pools (their waves then run only the
    // concurrent path: 10k invokers 33.9 vs 37.5 ms), spread over every wave for small pools, where concurrent walks
    // are long (1k invokers, 30 % concurrent: 553 vs 681 ms)
    p.deal = c->nm >= 4096 ? 1 : 2;
    if (env_opts().deal >= 0) p.deal = env_opts().deal;
    HIPCHK(c, c->d_lix.reserve((size_t)std::max<int64_t>(max_chunks, 1) * wl));
    p.rec = c->d_rec.p;
    p.lix = c->d_lix.p;
    HIPCHK(c, c->variant ? owgs_launch_prepass_narrow(&p, c->d_cstart.p, max_chunks, s)
                         : owgs_launch_prepass(&p, c->d_cstart.p, max_chunks, s));
    A.n_batches = n_batches;
    A.acq_off = acq_off;
    A.n_act = n_act;
    A.rec = c->d_rec.p;
    A.lix = c->d_lix.p;
    return OWGS_OK;
}

static int run_engine(owgs_ctx* c, OwgsEngineArgs& A, hipStream_t s, bool launch = true) {
    int rc = lds_check(c);
    if (rc) return rc;
    // the map's overflow exists only for concurrent actions: a context without any never allocates it
    if (c->any_conc || (A.feat & OWGS_F_CONC)) {
        const int64_t n_new = A.n_act - c->grp_a0;  // (a group launch indexes the whole stream from its first batch)
        rc = ensure_ovf(c, n_new, s);
        if (rc) return rc;
        ovf_add(c, n_new);
    }
    A.ovf = ovf_args(c);
    A.ct_tmp = c->d_ct_tmp.p;
    // walk cursors: one tagged word per action; the tags of this launch's batches must not repeat a stored tag
    if (A.n_batches >= 0x1FFFF) return c->fail(OWGS_ERANGE, "more than 131070 batches in one call");
    const size_t na = (size_t)std::max(A.n_actions, 1);
    if (c->d_gcur.n < na || c->cur_tag + A.n_batches + 1 > 0x1FFFF) {
        HIPCHK(c, c->d_gcur.reserve(na));
        HIPCHK(c, hipMemsetAsync(c->d_gcur.p, 0, c->d_gcur.n * sizeof(uint32_t), s));
        c->cur_tag = 0;
    }
    A.gcur = c->d_gcur.p;
    A.cur_tag0 = c->cur_tag;
    c->cur_tag += A.n_batches;
    // counters: two blocks used in turn; each launch zeroes the other one at its end (no fill launch per call)
    A.stats = c->d_stats.p + (size_t)c->stats_par * OWGS_NSTATS;
    A.stats_next = c->d_stats.p + (size_t)(c->stats_par ^ 1) * OWGS_NSTATS;
    c->stats_last = c->stats_par;
    c->stats_par ^= 1;
    if (!c->ev_engine[0]) {
        HIPCHK(c, hipEventCreate(&c->ev_engine[0]));
        HIPCHK(c, hipEventCreate(&c->ev_engine[1]));
    }
    // the engine specialisation: the map code when any registered action is concurrent (its entries, releases and
    // overflow can only come from such actions), the general pool / sequence code when the call needs it
    A.feat |= (c->any_conc ? OWGS_F_CONC : 0) | ((c->pool_mode != 0 || A.seq != nullptr) ? OWGS_F_GEN : 0);
    if (env_opts().feat_all) A.feat = OWGS_F_ALL;  // diagnostics: always the general engine
    A.geom = OWGS_GEOM_TAG(variant_wl(c));
    if (!launch) return OWGS_OK;  // owgs_replay_device_multi launches every shard's engine at once
    // the overflow's entry count for a later ensure_ovf: the engine stores it into a pinned probe slot as its last
    // step (no copy after the launch), read without a wait once the slot's event has passed
    int probe = -1;
    if (c->ovf_cap > 0) {
        const int rc = ovf_probe_slot(c, &probe);
        if (rc) return rc;
        if (probe >= 0) A.ovf_host = &c->h_ovf_cnt[probe];
    }
    HIPCHK(c, hipEventRecord(c->ev_engine[0], s));  // brackets exactly the engine launch (owgs_engine_ms)
    HIPCHK(c, launch_engine(c, &A, s));
    HIPCHK(c, hipEventRecord(c->ev_engine[1], s));
    c->ev_engine_valid = true;
    if (probe >= 0) {
        const int rc = ovf_probe_mark(c, probe, s);
        if (rc) return rc;
    }
    if (A.trace) {  // diagnostic timeline: raw u64 pairs, [waves][16384][2]
        HIPCHK(c, hipStreamSynchronize(s));
        std::vector<unsigned long long> h(c->d_trace.n);
        HIPCHK(c, hipMemcpy(h.data(), c->d_trace.p, h.size() * 8, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("OWGS_TRACE_FILE"), "wb")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
    return OWGS_OK;
}

// after a publish run in watch mode: Z of the watched pairs its decisions tried and failed (owgs_watch.hip).  d_act =
// the run's action handles (device), or null for explicit walks (d_xmeta / d_xslot of owgs_schedule_walks)
static int w_update(owgs_ctx* c, int32_t n, const int32_t* d_act, const int32_t* d_out, const uint8_t* d_fl,
                    hipStream_t s) {
    if (c->w_cap <= 0 || n <= 0) return OWGS_OK;
    const size_t na = std::max<size_t>(c->a_mem.size(), 1);
    const size_t had = c->w_D.n;
    HIPCHK(c, c->w_D.reserve(na));
    // zero between runs; a grown buffer is new memory (hipMalloc may hand back the freed address: compare sizes)
    if (c->w_D.n != had) HIPCHK(c, hipMemsetAsync(c->w_D.p, 0, c->w_D.n * 4, s));
    HIPCHK(c, c->w_L.reserve((size_t)n));
    HIPCHK(c, c->w_L2.reserve((size_t)n));
    HIPCHK(c, c->w_Lcnt.reserve(2));
    OwgsWUpdateArgs a{};
    a.n = n;
    a.act = d_act;
    a.act_meta = c->d_act_meta.p;
    a.act_slot = c->d_act_slot.p;
    a.xmeta = c->d_xmeta.p;
    a.xslot = c->d_xslot.p;
    a.out_inv = d_out;
    a.out_flags = d_fl;
    a.pool_mode = c->pool_mode;
    a.n_ids = c->n_ids;
    a.nm = c->nm;
    a.nb = c->nb;
    a.usable = c->d_usable.p;
    a.pool_words = c->d_pool_words.p;
    a.ct_keys = c->d_ct_keys.p;
    a.ovf = ovf_args(c);
    a.w = watch_args(c);
    a.D = c->w_D.p;
    a.L = c->w_L.p;
    a.L2 = c->w_L2.p;
    a.Lcnt = c->w_Lcnt.p;
    HIPCHK(c, owgs_launch_w_update(&a, s));
    return OWGS_OK;
}

static int check_err_word(owgs_ctx* c) {
    int32_t e = 0;
    HIPCHK(c, hipMemcpy(&e, c->d_err.p, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (e) {
        HIPCHK(c, hipMemset(c->d_err.p, 0, sizeof(int32_t)));
        if (e & OWGS_ERR_CTAB_FULL) return c->fail(OWGS_ENOMEM, "concurrency table full");
        if (e & OWGS_ERR_OPS) return c->fail(OWGS_ERANGE, "operationCount beyond the engine's range");
        if (e & OWGS_ERR_GEOM) return c->fail(OWGS_EDEVICE, "engine object and host disagree on the engine geometry");
        if (e & OWGS_ERR_INTERNAL) return c->fail(OWGS_EDEVICE, "engine invariant violated");
        if (e & OWGS_ERR_PERMITS) return c->fail(OWGS_ERANGE, "slot permits outside the engine's range [-2^29, 2^29) MB");
        if (e & OWGS_ERR_RELRISK)  // (stream mode only: the chunked engine applies such releases and flags FS:48-50)
            return c->fail(OWGS_ERANGE, "stream-mode replay stopped before a release that could overflow a slot's "
                                        "permits (ForcibleSemaphore.release FS:48-50): the rest of the stream is not "
                                        "applied; replay it with OWGS_SPEC_REPLAY=0");
        return c->fail(OWGS_EINVAL, "stream releases an activation that holds no slot (or a permit overflow)");
    }
    return OWGS_OK;
}

static bool registered(const owgs_ctx* c, int32_t n, const int32_t* action) {
    const int32_t na = (int32_t)c->a_mem.size();
    for (int32_t i = 0; i < n; ++i)
        if (action[i] < 0 || action[i] >= na || !c->a_live[action[i]]) return false;
    return true;
}

// Keys without live handles whose ids can be reused: no entry of the NestedSemaphore map (primary table, HBM overflow)
// and no watched pair names them any more -- the reference's map loses an entry at operationCount 0
// (NestedSemaphore.scala:109-111), so a key whose activations have all completed leaves nothing behind.  One scan
// over the tables on the device; keys still named stay pending for a later attempt.
static int reclaim_slots(owgs_ctx* c) {
    // (the large-state engine's map keeps the reference's empty entries, which never leave: its keys stay taken)
    if (c->pending_slots.empty() || c->large) return OWGS_OK;
    const size_t words = ((size_t)OWGS_MAX_SLOTKEYS + 32) / 32;
    std::vector<uint32_t> cand(words, 0u);
    size_t k = 0;
    for (int32_t sid : c->pending_slots)
        if (c->slot_uses[sid] == 0) cand[sid >> 5] |= 1u << (sid & 31);  // (re-registered keys dropped out)
    HIPCHK(c, upload(c->d_cand, cand.data(), words, c->stream));
    int32_t ovf_n = 0;
    if (c->ovf_cap > 0) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipMemcpy(&ovf_n, c->d_ovf_cnt.p, sizeof(ovf_n), hipMemcpyDeviceToHost));
    }
    HIPCHK(c, owgs_launch_slot_scan(c->d_ct_keys.p, ovf_n > 0 ? c->d_ovf.p : nullptr, ovf_n > 0 ? c->ovf_cap : 0,
                                    c->w_cap > 0 ? c->w_keys.p : nullptr, c->w_cap, c->w_cap > 0 ? c->w_wkey.p : nullptr,
                                    c->d_cand.p, c->stream));
    HIPCHK(c, hipMemcpyAsync(cand.data(), c->d_cand.p, words * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<int32_t> still;
    for (int32_t sid : c->pending_slots) {
        if (c->slot_uses[sid] != 0) continue;  // named by a live handle again
        if ((cand[sid >> 5] >> (sid & 31)) & 1u) {
            c->slot_ids.erase(c->slot_name[sid]);
            std::string().swap(c->slot_name[sid]);
            c->free_slots.push_back(sid);
            ++c->slot_epoch;
            ++k;
        } else {
            still.push_back(sid);
        }
    }
    c->pending_slots.swap(still);
    (void)k;
    return OWGS_OK;
}

// ---------------------------------------------------------------------------------------------- resident engine
// owgs_process_batch's small calls go to a resident engine (owgs_resident.hip) that keeps the slot state in LDS
// between calls.  Every other entry point reads or replaces that state, so it stops the engine first (the engine
// writes the state back to HBM and exits) -- OWGS_ENTER below; the next eligible call launches it again.
// after the engine's stream has drained: count an exit the lifetime bound caused (diagnostics)
static void res_reap(owgs_ctx* c) {
    if (__atomic_load_n(&c->res_ctl[OWGS_RES_STATE], __ATOMIC_ACQUIRE) == 2 &&
        __atomic_load_n(&c->res_ctl[OWGS_RES_WHY], __ATOMIC_ACQUIRE) == 2)
        ++c->res_n_life;
    c->res_ctl[OWGS_RES_STATE] = 0;
}
static int res_quiesce(owgs_ctx* c) {
    if (!c->res_alive) return OWGS_OK;
    __atomic_store_n(&c->res_ctl[OWGS_RES_BELL], -1, __ATOMIC_RELEASE);
    c->res_alive = false;
    HIPCHK(c, hipStreamSynchronize(c->res_stream));
    res_reap(c);
    if (c->w_cap > 0 && c->w_live <= 0) w_drop(c);  // the engine's calls took the last pairs out of W
    return OWGS_OK;
}

#define OWGS_ENTER(c)                             \
    do {                                          \
        (void)hipSetDevice((c)->cfg.device);      \
        const int q_ = res_quiesce(c);            \
        if (q_) return q_;                        \
    } while (0)

static size_t res_stage_bytes(const owgs_ctx* c) {
    const size_t img = owgs_resident_image_bytes(c->n_slots, c->n_ids);
    return img >= OWGS_LDS_BYTES ? 0 : std::min<size_t>(OWGS_LDS_BYTES - img, 64 * 1024) & ~(size_t)15;
}

// identity pools, a call the staging area holds (watched pairs included: the engine applies their releases and marks)
static bool res_eligible(const owgs_ctx* c, int32_t n_runs, int32_t NR, int32_t NP, bool has_seq) {
    if (env_opts().res <= 0 || c->pool_mode != 0 || c->large) return false;
    if (c->w_cap > 0 && env_opts().res_watch <= 0) return false;
    if ((int64_t)NR + NP > env_opts().res_max || NP + NR == 0) return false;
    if (c->n_slots > OWGS_MAX_SLOTS_CT || c->n_ids > c->n_slots || c->nm > (int32_t)OWGS_AM_POS_MASK ||
        c->nb > (int32_t)OWGS_AM_POS_MASK || c->a_mem.empty())
        return false;
    const size_t runs = ((size_t)n_runs + 4) & ~(size_t)3;
    const size_t in_b = 8 * runs + (4 * (size_t)NP + 16) + 2 * (4 * (size_t)NR + 16) + (has_seq ? 8 * (size_t)NP : 0);
    // + the records the engine gathers, cursors, outputs
    const size_t need = in_b + 16 + 16 * (size_t)NR + 16 * (size_t)NP + 8 * (size_t)NP + 16 + 5 * (size_t)NP +
                        (size_t)NR + 32;
    if (need > res_stage_bytes(c) || res_stage_bytes(c) < 4096) return false;
    // a map that may outgrow its overflow table during the call: the chained path grows it
    if (c->any_conc && c->res_alive && c->ovf_cap < ovf_need(c->ovf_used_ub, NP)) return false;
    return true;
}

// The resident engine's index of the watched pairs: per fqn@version key with watched pairs
// {slot + 1, first, count, primary action} in an open-addressing table, and the key's pairs {W index, walk step of the
// pair's invoker in the primary action's walk} sorted by step, so that a decision marks the pairs before its step by
// reading a prefix.  The primary action is the key's lowest live concurrent handle; another action of the key computes
// each pair's step itself.  Built at every launch (W, the pools and the actions only change while no engine runs).
static int res_w_index(owgs_ctx* c) {
    c->w_scap = 0;
    if (c->w_cap <= 0) return OWGS_OK;
    std::vector<uint32_t> keys((size_t)c->w_cap);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(keys.data(), c->w_keys.p, keys.size() * 4, hipMemcpyDeviceToHost));
    std::unordered_map<int32_t, std::vector<uint2>> by_slot;  // slot -> {W index, step}
    for (int32_t j = 0; j < c->w_cap; ++j) {
        const uint32_t k = keys[(size_t)j];
        if (k == 0u || k == OWGS_CT_TOMB) continue;
        by_slot[(int32_t)(k >> OWGS_CT_SLOT_SHIFT)].push_back(make_uint2((uint32_t)j, 0x7FFFFFFFu));
    }
    std::unordered_map<int32_t, int32_t> prim;
    for (size_t a = 0; a < c->a_mem.size(); ++a)
        if (c->a_live[a] && c->a_maxc[a] > 1 && by_slot.count(c->a_slot[a]) && !prim.count(c->a_slot[a]))
            prim[c->a_slot[a]] = (int32_t)a;
    auto inv_mod = [](int64_t x, int64_t n) {
        int64_t t = 0, nt = 1, r = n, nr = x % n;
        while (nr) {
            const int64_t q = r / nr;
            int64_t tmp = t - q * nt;
            t = nt;
            nt = tmp;
            tmp = r - q * nr;
            r = nr;
            nr = tmp;
        }
        return t < 0 ? t + n : t;
    };
    std::vector<uint2> list;
    std::vector<uint4> sidx;
    size_t scap = 16;
    while (scap < 2 * by_slot.size()) scap <<= 1;
    sidx.assign(scap, make_uint4(0u, 0u, 0u, 0u));
    for (auto& kv : by_slot) {
        const int32_t slot = kv.first;
        auto it = prim.find(slot);
        const int32_t pa = it == prim.end() ? -1 : it->second;  // (none: every decision of the key computes steps)
        if (pa >= 0 && (size_t)pa < c->res_meta.size() && !(c->res_meta[pa].y & (OWGS_AM_EMPTY | OWGS_AM_THROW))) {
            const uint32_t mx = c->res_meta[pa].x;
            const int64_t pool = (mx & OWGS_AM_POOL) ? 1 : 0, n = pool ? c->nb : c->nm;
            const int64_t base = pool ? c->n_ids - c->nb : 0, home = mx & OWGS_AM_POS_MASK;
            const int64_t step = (mx >> 15) & OWGS_AM_POS_MASK;
            const int64_t is = n > 1 ? inv_mod(step % n, n) : 0;
            for (uint2& e : kv.second) {
                const int64_t x = (int64_t)(keys[e.x] & 0x7FFFu) - 1, pos = x - base;
                if (n > 0 && pos >= 0 && pos < n) e.y = (uint32_t)(n > 1 ? ((pos - home + n) % n) * is % n : 0);
            }
            std::sort(kv.second.begin(), kv.second.end(), [](const uint2& a, const uint2& b) { return a.y < b.y; });
        }
        uint32_t h = 0;
        {  // ct_hash(slot + 1), as the device probes
            uint32_t k = (uint32_t)slot + 1u;
            k ^= k >> 16;
            k *= 0x7feb352dU;
            k ^= k >> 15;
            k *= 0x846ca68bU;
            k ^= k >> 16;
            h = k & (uint32_t)(scap - 1);
        }
        while (sidx[h].x != 0u) h = (h + 1u) & (uint32_t)(scap - 1);
        sidx[h] = make_uint4((uint32_t)slot + 1u, (uint32_t)list.size(), (uint32_t)kv.second.size(),
                             pa >= 0 ? (uint32_t)pa : 0xFFFFFFFFu);
        list.insert(list.end(), kv.second.begin(), kv.second.end());
    }
    if (list.empty()) list.push_back(make_uint2(0u, 0u));
    HIPCHK(c, c->d_w_sidx.reserve(scap));
    HIPCHK(c, c->d_w_list.reserve(list.size()));
    HIPCHK(c, hipMemcpy(c->d_w_sidx.p, sidx.data(), scap * sizeof(uint4), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_w_list.p, list.data(), list.size() * sizeof(uint2), hipMemcpyHostToDevice));
    c->w_scap = (int32_t)scap;
    return OWGS_OK;
}

static int res_launch(owgs_ctx* c) {
    if (!c->res_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->res_stream, hipStreamNonBlocking));
    if (!c->ev_res) HIPCHK(c, hipEventCreateWithFlags(&c->ev_res, hipEventDisableTiming));
    if (!c->res_ctl) {
        HIPCHK(c, hipHostMalloc((void**)&c->res_ctl, OWGS_RES_CTL_WORDS * sizeof(int32_t), hipHostMallocCoherent));
        memset(c->res_ctl, 0, OWGS_RES_CTL_WORDS * sizeof(int32_t));
    }
    if (c->any_conc) {  // the map's overflow, sized for this call (before the engine holds the table)
        const int rc = ensure_ovf(c, env_opts().res_max, c->stream);
        if (rc) return rc;
    }
    HIPCHK(c, c->d_ct_tmp.reserve((size_t)2 * OWGS_CTC));
    if (c->res_n_launches == 0) {  // (tests: start below the wrap limits)
        c->res_call = (int32_t)std::min<long long>(std::max<long long>(env_opts().res_call_base, 0), OWGS_RES_CALL_LIMIT);
        // (never backwards: a stream-mode replay may already have stored cursors under the generations up to here)
        const uint32_t base = (uint32_t)std::min<long long>(std::max<long long>(env_opts().res_gen_base, 0), 0xFFFFFFFFll);
        c->res_gen_seen = std::max(c->res_gen_seen, base);
    } else {
        c->res_call = 0;  // a fresh engine: the bell counts up from 0 again (it stays in [0, 2^31): -1 is the stop word)
    }
    {  // walk cursors: a new buffer starts at generation 0, below every generation a launch uses; a generation near
       // its 32-bit wrap starts over from 0 (every stored cursor cleared: an equal generation must mean this launch's)
        const size_t na = std::max<size_t>(c->a_mem.size(), 1);
        const bool wrap = (uint64_t)c->res_gen_seen + 2 >= OWGS_RES_GEN_LIMIT;
        if (c->d_res_cur.n < na || wrap) {
            if (c->d_res_cur.n < na) HIPCHK(c, c->d_res_cur.reserve(na + na / 2));
            HIPCHK(c, hipMemsetAsync(c->d_res_cur.p, 0, c->d_res_cur.n * sizeof(uint2), c->stream));
            if (wrap) c->res_gen_seen = 0;
        }
    }
    // the action meta the host writes into each call's records (as the device computed it) and the watched-pair
    // index: downloaded / rebuilt only when actions, pools or W changed since the last launch (a relaunch after a
    // chained call would otherwise pay a synchronised copy of every action's meta)
    const bool fresh = c->res_cache_seen == c->res_cache_epoch && c->res_meta.size() == c->a_mem.size();
    if (!fresh) {
        c->res_meta.resize(c->a_mem.size());
        if (!c->res_meta.empty()) {
            HIPCHK(c, hipMemcpyAsync(c->res_meta.data(), c->d_act_meta.p, c->res_meta.size() * sizeof(uint2),
                                     hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
        }
    }
    if (!fresh || (c->w_cap > 0) != (c->w_scap > 0)) {
        const int rc = res_w_index(c);
        if (rc) return rc;
        c->res_cache_seen = c->res_cache_epoch;
    }
    // the state in HBM must be current: the resident stream waits for the context's stream and its last async call
    HIPCHK(c, hipEventRecord(c->ev_res, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->res_stream, c->ev_res, 0));
    if (c->tail_valid && c->tail_stream != c->stream) HIPCHK(c, hipStreamWaitEvent(c->res_stream, c->ev_tail, 0));
    OwgsResArgs a{};
    a.permits = c->d_permits.p;
    a.n_slots = c->n_slots;
    a.usable = c->d_usable.p;
    a.n_ids = c->n_ids;
    a.nm = c->nm;
    a.nb = c->nb;
    a.ct_keys = c->d_ct_keys.p;
    a.ct_vals = c->d_ct_vals.p;
    a.ct_tmp = c->d_ct_tmp.p;
    a.ovf = ovf_args(c);
    a.act_meta = c->d_act_meta.p;
    a.act_slot = c->d_act_slot.p;
    a.n_actions = (int32_t)c->a_mem.size();
    a.rng_seed = c->cfg.rng_seed;
    a.err = c->d_err.p;
    a.ctl = c->res_ctl;
    a.in = c->res_in;
    a.out = c->res_out;
    a.stage_bytes = (int32_t)res_stage_bytes(c);
    a.last_call = c->res_call;
    a.cur = c->d_res_cur.p;  // (dropping them measured slower: drains inside a batch's publishes keep the generation)
    a.gen_base = ++c->res_gen_seen;  // above every generation stored by earlier launches
    a.idle_ticks = env_opts().res_idle_us * 100;  // s_memrealtime: 100 MHz
    a.life_ticks = std::max(0ll, env_opts().res_life_us) * 100;
    a.spec = std::max(0, env_opts().res_spec);
    a.cspec = std::max(0, env_opts().res_cspec);
    a.cspec_pre = std::max(0, env_opts().res_cspec_pre);
    a.hsplit = std::max(0, std::min(3, env_opts().res_split));
    a.prespec = env_opts().res_pre;
    a.w = watch_args(c);
    a.w_sidx = c->d_w_sidx.p;
    a.w_scap = c->w_scap;
    a.w_list = c->d_w_list.p;
    if (c->w_cap > 0) c->res_ctl[OWGS_RES_WLIVE] = c->w_live;
    volatile int32_t* ctl = c->res_ctl;
    ctl[OWGS_RES_STATE] = 0;
    ctl[OWGS_RES_DONE] = c->res_call;
    __atomic_store_n(&c->res_ctl[OWGS_RES_BELL], c->res_call, __ATOMIC_RELEASE);
    const size_t lds = owgs_resident_image_bytes(c->n_slots, c->n_ids) + (size_t)a.stage_bytes;
    HIPCHK(c, owgs_launch_resident(&a, lds, c->res_stream));
    c->res_alive = true;
    ++c->res_n_launches;
    return OWGS_OK;
}

// one owgs_process_batch call through the resident engine; *served = 0: refused untouched (the caller takes the chain)
static int res_process(owgs_ctx* c, int32_t n_runs, const int32_t* rel_off, const int32_t* rel_invoker,
                       const int32_t* rel_action, uint8_t* rel_flags, const int32_t* pub_off, const int32_t* pub_action,
                       const uint64_t* seq, uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags, int* served) {
    *served = 0;
    const auto th0 = std::chrono::steady_clock::now();
    const int32_t NR = rel_off[n_runs], NP = pub_off[n_runs];
    // the call's input block (16-byte aligned parts): rel_off | pub_off | publish words (action | rank << 17 |
    // shared << 23) | release invokers | release actions | seq.  Handles only: the engine gathers each record's
    // action meta and slot key from HBM, so a call of up to ~1000 jobs crosses PCIe in the engine's first 4 KB read
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t b_poff = al(4 * ((size_t)n_runs + 1)), b_aid = b_poff + al(4 * ((size_t)n_runs + 1));
    const size_t b_rel = b_aid + al(4 * (size_t)NP);   // release invokers
    const size_t b_pub = b_rel + al(4 * (size_t)NR);   // release actions
    const size_t b_seq = b_pub + al(4 * (size_t)NR);
    const size_t in_bytes = al(b_seq + (seq ? 8 * (size_t)NP : 0));
    const size_t o_fl = 4 * (size_t)NP, o_rfl = o_fl + NP, out_bytes = al(o_rfl + NR) + 16;
    if (std::max<size_t>(in_bytes, 4096) > c->res_in_cap || out_bytes > c->res_out_cap) {  // (the engine holds the
        const int q = res_quiesce(c);                                                        // buffers' addresses)
        if (q) return q;
        if (std::max<size_t>(in_bytes, 4096) > c->res_in_cap) {
            if (c->res_in) (void)hipHostFree(c->res_in);
            c->res_in = nullptr;
            c->res_in_cap = 0;
            const size_t cap = std::max<size_t>(2 * in_bytes, 64 * 1024);
            HIPCHK(c, hipHostMalloc((void**)&c->res_in, cap, hipHostMallocCoherent));
            c->res_in_cap = cap;
        }
        if (out_bytes > c->res_out_cap) {
            if (c->res_out) (void)hipHostFree(c->res_out);
            c->res_out = nullptr;
            c->res_out_cap = 0;
            const size_t cap = std::max<size_t>(2 * out_bytes, 32 * 1024);
            HIPCHK(c, hipHostMalloc((void**)&c->res_out, cap, hipHostMallocCoherent));
            c->res_out_cap = cap;
        }
    }
    // the doorbell and the cursor generation stay below their limits: an engine near either is stopped (it writes
    // the state back) and the relaunch below starts both over
    if (c->res_alive && (c->res_call >= OWGS_RES_CALL_LIMIT - 8 ||
                         (uint64_t)c->res_gen_seen + (uint64_t)n_runs + 2 >= OWGS_RES_GEN_LIMIT)) {
        const int q = res_quiesce(c);
        if (q) return q;
    }
    if (!c->res_alive) {
        const int rc = res_launch(c);
        if (rc) return rc;
    }
    char* B = (char*)c->res_in;
    memcpy(B, rel_off, 4 * ((size_t)n_runs + 1));
    memcpy(B + b_poff, pub_off, 4 * ((size_t)n_runs + 1));
    if (NR) {
        memcpy(B + b_rel, rel_invoker, 4 * (size_t)NR);
        memcpy(B + b_pub, rel_action, 4 * (size_t)NR);
    }
    uint64_t rsum = 0;
    for (int32_t j = 0; j < NR; ++j)
        if (rel_invoker[j] >= 0 && rel_invoker[j] < c->n_slots) rsum += (uint64_t)c->a_mem[rel_action[j]];
    uint32_t* Q = (uint32_t*)(B + b_aid);
    // per chunk of 64 publishes of a run (the engine's speculation unit): each publish's rank among the chunk's
    // publishes of its action, and whether an earlier concurrent publish of the chunk has its fqn@version key under
    // another action (owgs_resident.hip, RES_RANK_SHIFT / RES_SHARED)
    {
        struct Tab {  // 128-entry open addressing, cleared by its used list
            uint32_t k[128];
            int32_t v[128];
            int32_t w[128];
            uint8_t used[128];
            int32_t list[64];
            int n = 0;
            Tab() { memset(used, 0, sizeof(used)); }
            int find(uint32_t key) {
                uint32_t h = (key * 2654435761u) >> 25;
                while (used[h] && k[h] != key) h = (h + 1) & 127;
                if (!used[h]) {
                    used[h] = 1;
                    k[h] = key;
                    v[h] = 0;
                    w[h] = -1;
                    list[n++] = (int)h;
                }
                return (int)h;
            }
            void clear() {
                for (int i = 0; i < n; ++i) used[list[i]] = 0;
                n = 0;
            }
        };
        static thread_local Tab ta, ts;
        for (int32_t r = 0; r < n_runs; ++r)
            for (int32_t c0 = pub_off[r]; c0 < pub_off[r + 1]; c0 += 64) {
                const int32_t c1 = std::min(c0 + 64, pub_off[r + 1]);
                for (int32_t i = c0; i < c1; ++i) {
                    const int32_t a = pub_action[i];
                    const int ha = ta.find((uint32_t)a);
                    uint32_t wd = (uint32_t)a | ((uint32_t)ta.v[ha]++ << 17);
                    const uint32_t my = c->res_meta[a].y;
                    if (!(my & (OWGS_AM_EMPTY | OWGS_AM_THROW)) && c->a_maxc[a] > 1) {
                        const int hs = ts.find((uint32_t)c->a_slot[a]);
                        if (ts.w[hs] < 0) ts.w[hs] = a;                     // first concurrent action of the key
                        else if (ts.w[hs] != a) ts.v[hs] = 1;                // a second action: later ones are shared
                        if (ts.w[hs] != a || ts.v[hs]) wd |= 1u << 23;
                    }
                    Q[i] = wd;
                }
                ta.clear();
                ts.clear();
            }
    }
    if (seq && NP) memcpy(B + b_seq, seq, 8 * (size_t)NP);
    volatile int32_t* H = c->res_ctl + OWGS_RES_HDR;
    const int32_t hdr[14] = {n_runs, NR, NP, seq ? 1 : 0, (int32_t)(uint32_t)seq_base, (int32_t)(uint32_t)(seq_base >> 32),
                             (int32_t)b_poff, (int32_t)b_rel, (int32_t)b_pub, (int32_t)b_seq, (int32_t)in_bytes,
                             (int32_t)(uint32_t)rsum, (int32_t)(uint32_t)(rsum >> 32), (int32_t)b_aid};
    for (int k = 0; k < 14; ++k) H[k] = hdr[k];
    const auto th1 = std::chrono::steady_clock::now();
    for (int attempt = 0;; ++attempt) {
        const int32_t k = ++c->res_call;
        __atomic_store_n(&c->res_ctl[OWGS_RES_BELL], k, __ATOMIC_RELEASE);
        const auto t0 = std::chrono::steady_clock::now();
        bool exited = false;
        for (long spin = 0;; ++spin) {
            if (__atomic_load_n(&c->res_ctl[OWGS_RES_DONE], __ATOMIC_ACQUIRE) == k) break;
            if (__atomic_load_n(&c->res_ctl[OWGS_RES_STATE], __ATOMIC_ACQUIRE) == 2 &&
                __atomic_load_n(&c->res_ctl[OWGS_RES_DONE], __ATOMIC_ACQUIRE) != k) {
                exited = true;  // it went idle and wrote the state back before it saw this call
                break;
            }
            if ((spin & 1023) == 1023 &&
                std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                c->res_alive = false;  // (nothing to wait for safely: the context is unusable from here)
                return c->fail(OWGS_EDEVICE, "resident engine did not answer");
            }
            __builtin_ia32_pause();
        }
        if (!exited) break;
        HIPCHK(c, hipStreamSynchronize(c->res_stream));
        res_reap(c);
        c->res_alive = false;
        if (attempt >= 3) return c->fail(OWGS_EDEVICE, "resident engine exits before serving a call");
        const int rc = res_launch(c);
        if (rc) return rc;
    }
    const int32_t res = __atomic_load_n(&c->res_ctl[OWGS_RES_RESULT], __ATOMIC_ACQUIRE);
    const int bail = res & 0xFF, e = res >> 8;
    {
        const auto th2 = std::chrono::steady_clock::now();
        c->res_host_ns[0] += std::chrono::duration_cast<std::chrono::nanoseconds>(th1 - th0).count();
        c->res_host_ns[1] += std::chrono::duration_cast<std::chrono::nanoseconds>(th2 - th1).count();
    }
    if (bail) {
        ++c->res_n_bails;
        return OWGS_OK;  // nothing applied: the chained path takes the call
    }
    ++c->res_n_calls;
    if (c->w_cap > 0) {  // watched pairs left (W itself is dropped once the engine has stopped: res_quiesce)
        c->w_live = __atomic_load_n(&c->res_ctl[OWGS_RES_WLIVE], __ATOMIC_ACQUIRE);
        ++c->res_n_watch_calls;
    }
    c->res_gen_seen = (uint32_t)__atomic_load_n(&c->res_ctl[OWGS_RES_GEN], __ATOMIC_ACQUIRE);
    for (int k = 0; k < OWGS_RES_NPROF; ++k) c->res_prof[k] += (uint32_t)c->res_ctl[OWGS_RES_PROF + k];
    c->res_used_max = std::max<int64_t>(c->res_used_max, c->res_ctl[OWGS_RES_USED]);
    c->res_tombs_max = std::max<int64_t>(c->res_tombs_max, c->res_ctl[OWGS_RES_TOMBS]);
    if (c->any_conc) ovf_add(c, NP);
    if (NP) {
        memcpy(out_invoker, c->res_out, 4 * (size_t)NP);
        memcpy(out_flags, c->res_out + o_fl, (size_t)NP);
    }
    if (NR && rel_flags) memcpy(rel_flags, c->res_out + o_rfl, (size_t)NR);
    *served = 1;
    if (e) {
        if (e & OWGS_ERR_CTAB_FULL) return c->fail(OWGS_ENOMEM, "concurrency table full");
        if (e & OWGS_ERR_OPS) return c->fail(OWGS_ERANGE, "operationCount beyond the engine's range");
        if (e & OWGS_ERR_INTERNAL) return c->fail(OWGS_EDEVICE, "engine invariant violated");
        if (e & OWGS_ERR_PERMITS) return c->fail(OWGS_ERANGE, "slot permits outside the engine's range [-2^29, 2^29) MB");
        return c->fail(OWGS_EINVAL, "call names an unknown action");
    }
    return OWGS_OK;
}

// ---------------------------------------------------------------------------------------------- large-state engine
// owgs_seq.hip: contexts whose state no on-chip geometry holds (owgs_limits), or with maxConcurrent > OWGS_MAX_CONC.
// Identity pools; every call through it is synchronous (the host reads where the kernel stopped to grow the map).
#define OWGS_NOT_LARGE(c)                                                                                   \
    do {                                                                                                  \
        if ((c)->large)                                                                                   \
            return (c)->fail(OWGS_ERANGE, "not available for a state beyond owgs_limits (large-state engine)"); \
    } while (0)

static bool large_fits(int32_t n_ids, int32_t nm, int32_t nb) {
    return n_ids <= OWGS_SEQ_MAX_WORDS * 32 && nm <= owgs_coprime_max() && nb <= owgs_coprime_max();
}

static OwgsSeqArgs seq_args(owgs_ctx* c) {
    OwgsSeqArgs S{};
    S.permits = c->d_permits.p;
    S.n_slots = c->n_slots;
    S.usable = c->d_usable.p;
    S.n_ids = c->n_ids;
    S.nm = c->nm;
    S.nb = c->nb;
    S.msteps = c->d_steps.p;
    S.n_msteps = (int32_t)c->msteps.size();
    S.bsteps = c->d_steps.p + c->steps_stride;
    S.n_bsteps = (int32_t)c->bsteps.size();
    S.act_hash = c->d_act_hash.p;
    S.act_mem = c->d_act_mem.p;
    S.act_maxc = c->d_act_maxc.p;
    S.act_slot = c->d_act_slot.p;
    S.act_bb = c->d_act_bb.p;
    S.cur = c->q_cur.p;
    S.n_actions = c->q_cur.p ? (int32_t)c->a_mem.size() : 0;
    S.gen0 = c->q_gen;
    S.map = c->q_map.p;
    S.map_cap = c->q_cap;
    S.map_filled = c->q_filled.p;
    S.rng_seed = c->cfg.rng_seed;
    S.state = c->q_state.p;
    S.err = c->d_err.p;
    return S;
}

// the map keeps `room` more entries under half its capacity: read its fill, grow (rehash live entries) if needed
static int seq_reserve(owgs_ctx* c, int64_t room, hipStream_t s) {
    HIPCHK(c, c->q_state.reserve(16));
    if (!c->q_filled.p) {
        HIPCHK(c, c->q_filled.reserve(1));
        HIPCHK(c, hipMemsetAsync(c->q_filled.p, 0, 4, s));
    }
    int32_t filled = 0;
    if (c->q_cap > 0) {
        HIPCHK(c, hipMemcpyAsync(&filled, c->q_filled.p, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        if ((int64_t)c->q_cap >= 2 * ((int64_t)filled + room)) return OWGS_OK;
    }
    int64_t cap = (int64_t)1 << 16;
    while (cap < 4 * ((int64_t)filled + room)) cap <<= 1;
    if (cap > ((int64_t)1 << 30)) return c->fail(OWGS_ENOMEM, "NestedSemaphore map beyond 2^30 entries");
    DevBuf<uint4> nt;
    HIPCHK(c, nt.reserve((size_t)cap));
    HIPCHK(c, hipMemsetAsync(nt.p, 0, (size_t)cap * sizeof(uint4), s));
    HIPCHK(c, hipMemsetAsync(c->q_filled.p, 0, 4, s));  // (the rehash counts the live entries again)
    if (c->q_cap > 0) {
        OwgsSeqArgs S = seq_args(c);
        S.map = nt.p;
        S.map_cap = (int32_t)cap;
        HIPCHK(c, owgs_launch_seq_rehash(c->q_map.p, c->q_cap, &S, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    c->q_map.release();
    c->q_map = nt;
    nt.p = nullptr;
    c->q_cap = (int32_t)cap;
    return OWGS_OK;
}

// the context switches to the large-state engine: the on-chip map's entries (and the empty entries watched pairs stand
// for) move into the large map; the on-chip map and W are then unused
static int seq_migrate(owgs_ctx* c) {
    hipStream_t s = c->stream;
    int32_t ovf_n = 0;
    if (c->ovf_cap > 0) {
        HIPCHK(c, hipStreamSynchronize(s));
        HIPCHK(c, hipMemcpy(&ovf_n, c->d_ovf_cnt.p, sizeof(ovf_n), hipMemcpyDeviceToHost));
    }
    int rc = seq_reserve(c, (int64_t)OWGS_CTC + ovf_n + std::max(c->w_cap, 0) + 4096, s);
    if (rc) return rc;
    OwgsSeqArgs S = seq_args(c);
    if (c->d_ct_keys.p || (c->w_cap > 0))
        HIPCHK(c, owgs_launch_seq_migrate(c->d_ct_keys.p, c->d_ct_vals.p, c->d_ct_keys.p ? OWGS_CTC : 0,
                                          ovf_n > 0 ? c->d_ovf.p : nullptr, c->ovf_cap, c->w_cap > 0 ? c->w_keys.p : nullptr,
                                          c->w_vals.p, c->w_cap, &S, s));
    HIPCHK(c, hipStreamSynchronize(s));
    rc = check_err_word(c);
    if (rc) return rc;
    w_drop(c);
    return reset_ctab(c);
}

// runs through the large-state engine (S: its runs, releases, publishes, outputs); resumes after map growth
static int seq_run(owgs_ctx* c, const OwgsSeqArgs& S0, hipStream_t s) {
    const int64_t room = 2 * ((int64_t)std::max(c->nm, c->nb) + 2) + 4096;
    // walk cursors: one per action, tagged with a generation that no earlier call used (state changes between calls
    // -- health, cluster size, restores -- need no invalidation); all zero again before the counter could wrap
    const size_t na = c->a_mem.size();
    if (na > 0 && c->q_cur.n < na) {
        DevBuf<uint4> nc;
        HIPCHK(c, nc.reserve(na + na / 2 + 64));
        HIPCHK(c, hipMemsetAsync(nc.p, 0, nc.n * sizeof(uint4), s));
        HIPCHK(c, hipStreamSynchronize(s));
        c->q_cur.release();
        c->q_cur = nc;
        nc.p = nullptr;
        nc.n = 0;
    }
    if (c->q_gen > 0xF0000000u) {
        if (c->q_cur.p) HIPCHK(c, hipMemsetAsync(c->q_cur.p, 0, c->q_cur.n * sizeof(uint4), s));
        c->q_gen = 1;
    }
    uint32_t gen = c->q_gen;
    for (int resume = 0;; resume = 1) {
        const int rc = seq_reserve(c, room, s);
        if (rc) return rc;
        OwgsSeqArgs S = S0;
        S.cur = na > 0 ? c->q_cur.p : nullptr;
        S.n_actions = (int32_t)na;
        S.gen0 = gen;
        S.map = c->q_map.p;
        S.map_cap = c->q_cap;
        S.map_filled = c->q_filled.p;
        S.state = c->q_state.p;
        S.resume = resume;
        HIPCHK(c, owgs_launch_seq(&S, s));
        int32_t st[16] = {0};
        HIPCHK(c, hipMemcpyAsync(st, c->q_state.p, sizeof(st), hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        c->q_spec += st[6];  // (decisions the launch kept from its speculation / decided alone)
        c->q_alone += st[7];
        for (int k = 0; k < 4; ++k) c->q_cyc[k] += (uint64_t)(uint32_t)st[8 + 2 * k] | ((uint64_t)(uint32_t)st[9 + 2 * k] << 32);
        gen = (uint32_t)st[5];  // (a resumed launch continues the generation it stopped in)
        if (st[0] == 0) break;
    }
    c->q_gen = gen + 1u;
    return check_err_word(c);
}

// runs of explicit (host) releases and publishes, as owgs_process_batch / owgs_publish_batch / owgs_release_batch
static int seq_host_runs(owgs_ctx* c, int32_t n_runs, const int32_t* rel_off, const int32_t* rel_inv,
                         const int32_t* rel_act, uint8_t* rel_flags, const int32_t* pub_off, const int32_t* pub_act,
                         const uint64_t* seq, uint64_t seq_base, int32_t* out_inv, uint8_t* out_flags) {
    hipStream_t s = c->stream;
    const int32_t NR = rel_off[n_runs], NP = pub_off[n_runs];
    std::vector<int64_t> offs((size_t)2 * (n_runs + 1));
    for (int32_t r = 0; r <= n_runs; ++r) {
        offs[r] = rel_off[r];
        offs[n_runs + 1 + r] = pub_off[r];
    }
    HIPCHK(c, upload(c->g_off, offs.data(), offs.size(), s));
    if (NR) {
        HIPCHK(c, upload(c->d_b, rel_inv, (size_t)NR, s));
        HIPCHK(c, upload(c->d_c, rel_act, (size_t)NR, s));
        HIPCHK(c, c->d_rflags.reserve((size_t)NR));
    }
    if (NP) {
        HIPCHK(c, upload(c->d_a, pub_act, (size_t)NP, s));
        HIPCHK(c, c->d_out.reserve((size_t)NP));
        HIPCHK(c, c->d_flags.reserve((size_t)NP));
        if (seq) HIPCHK(c, upload(c->d_seq, (const u64*)seq, (size_t)NP, s));
    }
    OwgsSeqArgs S = seq_args(c);
    S.n_runs = n_runs;
    S.rel_off = c->g_off.p;
    S.pub_off = c->g_off.p + n_runs + 1;
    S.rel_inv = c->d_b.p;
    S.rel_act = c->d_c.p;
    S.rel_flags = NR ? c->d_rflags.p : nullptr;
    S.pub_act = c->d_a.p;
    S.seq = (seq && NP) ? c->d_seq.p : nullptr;
    S.seq_base = seq_base;
    S.out_inv = c->d_out.p;
    S.out_flags = c->d_flags.p;
    const int rc = seq_run(c, S, s);
    if (NP) {
        HIPCHK(c, hipMemcpyAsync(out_inv, c->d_out.p, (size_t)NP * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(out_flags, c->d_flags.p, (size_t)NP, hipMemcpyDeviceToHost, s));
    }
    if (NR && rel_flags) HIPCHK(c, hipMemcpyAsync(rel_flags, c->d_rflags.p, (size_t)NR, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return rc;
}

// a device-resident stream's batches (releases by activation: invoker out_inv[aid], action act[aid])
static int seq_device_runs(owgs_ctx* c, int32_t n_runs, const int64_t* d_rel_off, const int64_t* d_pub_off,
                           const int32_t* act, const int64_t* rel_aid, uint64_t seq_base, int32_t* out_inv,
                           uint8_t* out_flags, uint8_t* rel_flags, hipStream_t s) {
    OwgsSeqArgs S = seq_args(c);
    S.n_runs = n_runs;
    S.rel_off = d_rel_off;
    S.pub_off = d_pub_off;
    S.rel_aid = rel_aid;
    S.dec_inv = out_inv;
    S.dec_act = act;
    S.rel_flags = rel_flags;
    S.pub_act = act;
    S.seq_base = seq_base;
    S.out_inv = out_inv;
    S.out_flags = out_flags;
    return seq_run(c, S, s);
}

// times one ABI call, entry to return, into c->last_call_ns (the latency the JNI shim sees, without the host
// language's call overhead)
struct CallTimer {
    owgs_ctx* c;
    std::chrono::steady_clock::time_point t0;
    explicit CallTimer(owgs_ctx* c_) : c(c_), t0(std::chrono::steady_clock::now()) {}
    ~CallTimer() {
        if (c) c->last_call_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
};

extern "C" {

int owgs_abi_version(void) { return OWGS_ABI_VERSION; }

// Diagnostics: both engine objects refuse a launch prepared for the other geometry before anything runs (the launch
// wrappers compare the geometry tag; no device is touched, so this runs without a GPU).  OWGS_OK when every wrapper
// refused, OWGS_EDEVICE naming the one that did not.
int owgs_geometry_selfcheck(void) {
    OwgsEngineArgs A;
    memset(&A, 0, sizeof(A));
    OwgsPrepassArgs p{};
    p.cw = 1;
    for (int v = 0; v < 2; ++v) {
        // the tag of the OTHER geometry (what a host sized for it would send)
        A.geom = p.geom = OWGS_GEOM_TAG(v ? OWGS_WL : OWGS_WL_NARROW);
        const hipError_t e1 = v ? owgs_launch_engine_narrow(&A, nullptr) : owgs_launch_engine(&A, nullptr);
        const hipError_t e2 = v ? owgs_launch_engine_multi_narrow(&A, 1, nullptr) : owgs_launch_engine_multi(&A, 1, nullptr);
        const hipError_t e3 = v ? owgs_launch_prepass_narrow(&p, nullptr, 1, nullptr) : owgs_launch_prepass(&p, nullptr, 1, nullptr);
        if (e1 != hipErrorInvalidValue || e2 != hipErrorInvalidValue || e3 != hipErrorInvalidValue) return OWGS_EDEVICE;
    }
    return OWGS_OK;
}

int owgs_limits(int32_t* max_invokers, int32_t* max_slots) {
    // identity pools (the largest on-chip state per invoker: permits + usable bit + prefix counts): the largest
    // invoker count whose LDS image fits, found by bisection over the layout itself
    int32_t lo = 0, hi = OWGS_MAX_SLOTS_CT;
    while (lo < hi) {
        const int32_t mid = lo + (hi - lo + 1) / 2;
        if (engine_variant(mid, 0, mid, mid, mid) >= 0) lo = mid;
        else hi = mid - 1;
    }
    if (max_invokers) *max_invokers = lo;
    if (max_slots) *max_slots = lo;
    return OWGS_OK;
}

int owgs_create(const owgs_config* cfg, owgs_ctx** out) {
    if (!cfg || !out) return OWGS_EINVAL;
    *out = nullptr;
    owgs_ctx* c = new (std::nothrow) owgs_ctx();
    if (!c) return OWGS_ENOMEM;
    c->cfg = *cfg;
    // SCPB:467-468
    c->mf = std::max(0.0, std::min(1.0, cfg->managed_fraction));
    c->bf = std::max(1.0 - c->mf, std::min(1.0, cfg->blackbox_fraction));
    c->cluster = 1;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0 || cfg->device < 0 || cfg->device >= ndev) {
        delete c;
        return OWGS_EDEVICE;
    }
    if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return OWGS_EDEVICE;
    }
    if (c->d_ct_keys.reserve(OWGS_CTC) || c->d_ct_vals.reserve(OWGS_CTC) || c->d_ct_tmp.reserve(2 * OWGS_CTC) ||
        c->d_stats.reserve(2 * OWGS_NSTATS) ||
        c->d_err.reserve(1) || c->d_clast.reserve(1) || c->d_permits.reserve(1)) {
        owgs_destroy(c);
        return OWGS_ENOMEM;
    }
    if (reset_ctab(c) || hipMemset(c->d_err.p, 0, sizeof(int32_t)) != hipSuccess ||
        hipMemset(c->d_clast.p, 0, sizeof(int32_t)) != hipSuccess ||
        hipMemset(c->d_stats.p, 0, 2 * OWGS_NSTATS * sizeof(u64)) != hipSuccess) {
        owgs_destroy(c);
        return OWGS_EDEVICE;
    }
    int rc = rebuild_pools(c);
    if (rc) {
        owgs_destroy(c);
        return rc;
    }
    if (cfg->cluster_size > 1) owgs_update_cluster(c, cfg->cluster_size);
    (void)hipStreamSynchronize(c->stream);
    *out = c;
    return OWGS_OK;
}

void owgs_destroy(owgs_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->cfg.device);
    (void)res_quiesce(c);
    if (c->res_stream) (void)hipStreamDestroy(c->res_stream);
    c->res_stream = nullptr;
    if (c->ev_res) (void)hipEventDestroy(c->ev_res);
    c->ev_res = nullptr;
    if (c->res_ctl) (void)hipHostFree(c->res_ctl);
    if (c->res_in) (void)hipHostFree(c->res_in);
    if (c->res_out) (void)hipHostFree(c->res_out);
    c->res_ctl = c->res_in = nullptr;
    c->res_out = nullptr;
    c->d_res_cur.release();
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    DevBuf<int32_t>* i32s[] = {&c->d_permits, &c->d_pool_words, &c->d_hlist, &c->d_act_slot, &c->d_act_hash,
                               &c->d_act_mem,  &c->d_act_maxc,   &c->d_steps,  &c->d_cpx,     &c->d_err,
                               &c->d_a,        &c->d_b,          &c->d_c,      &c->d_d,        &c->d_out,
                               &c->d_cstart,   &c->d_relx,       &c->d_relcnt, &c->d_xslot,  &c->s_permits};
    for (auto* b : i32s) b->release();
    DevBuf<uint32_t>* u32s[] = {&c->d_usable, &c->d_ct_keys, &c->d_ct_vals, &c->d_ct_tmp, &c->s_ct_keys, &c->s_ct_vals};
    for (auto* b : u32s) b->release();
    c->d_act_bb.release();
    c->q_map.release();
    c->q_filled.release();
    c->q_state.release();
    c->q_cur.release();
    c->q_look.release();
    c->d_act_cok.release();
    c->d_act_meta.release();
    c->d_stats.release();
    c->d_margs.release();
    c->d_ovf.release();
    c->s_ovf.release();
    c->d_ovf_rc.release();
    c->d_ovf_touched.release();
    c->d_ovf_cnt.release();
    if (c->h_margs) (void)hipHostFree(c->h_margs);
    c->h_margs = nullptr;
    if (c->h_ovf_cnt) (void)hipHostFree(c->h_ovf_cnt);
    c->h_ovf_cnt = nullptr;
    for (int k = 0; k < owgs_ctx::OVF_PROBES; ++k) {
        if (c->ev_ovf[k]) (void)hipEventDestroy(c->ev_ovf[k]);
        c->ev_ovf[k] = nullptr;
    }
    if (c->ev_status) (void)hipEventDestroy(c->ev_status);
    c->ev_status = nullptr;
    if (c->ev_tail) (void)hipEventDestroy(c->ev_tail);
    c->ev_tail = nullptr;
    if (c->ev_margs) (void)hipEventDestroy(c->ev_margs);
    c->ev_margs = nullptr;
    c->d_off.release();
    c->d_flags.release();
    c->d_rflags.release();
    c->d_seq.release();
    c->d_rel.release();
    c->d_rec.release();
    c->d_lix.release();
    c->d_gcur.release();
    c->d_trace.release();
    c->d_rel_rec.release();
    c->d_xmeta.release();
    c->t_tw.release();
    c->t_tk.release();
    c->t_tv.release();
    c->t_owner.release();
    c->k_key.release();
    c->k_info.release();
    c->k_state.release();
    c->k_kind.release();
    c->k_oflags.release();
    c->k_bytes.release();
    c->k_cfl.release();
    DevBuf<int32_t>* ks[] = {&c->k_inst, &c->k_slot, &c->k_tick, &c->k_r0, &c->k_r1, &c->k_r2, &c->k_r3, &c->k_act};
    for (auto* b : ks) b->release();
    c->k_off.release();
    c->k_aid.release();
    c->k_cnt.release();
    DevBuf<char>* mc[] = {&c->m_ta, &c->m_tb, &c->m_rci, &c->m_tid, &c->m_content, &c->m_trace, &c->m_out};
    for (auto* b : mc) b->release();
    DevBuf<int64_t>* m64[] = {&c->m_ta_off, &c->m_tb_off, &c->m_tid_off, &c->m_tid_start, &c->m_content_off,
                              &c->m_trace_off, &c->m_len, &c->m_len_sorted, &c->m_out_off};
    for (auto* b : m64) b->release();
    DevBuf<int32_t>* m32[] = {&c->m_inv, &c->m_tmpl, &c->m_bad, &c->m_order, &c->m_iota, &c->m_cnt, &c->m_topic};
    for (auto* b : m32) b->release();
    c->m_key.release();
    c->m_key_sorted.release();
    c->m_aid.release();
    c->m_cause.release();
    c->m_flags.release();
    c->m_temp.release();
    DevBuf<uint32_t>* wu[] = {&c->w_keys, &c->w_vals, &c->s_w_keys, &c->s_w_vals};
    for (auto* b : wu) b->release();
    DevBuf<int32_t>* wi[] = {&c->w_cnt, &c->w_wkey, &c->w_D, &c->w_L, &c->w_Lcnt, &c->w_rel, &c->s_w_wkey};
    for (auto* b : wi) b->release();
    c->w_L2.release();
    c->w_off.release();
    c->w_rfl.release();
    if (c->h_pin) (void)hipHostFree(c->h_pin);
    if (c->h_pout) (void)hipHostFree(c->h_pout);
    c->h_pin = c->h_pout = nullptr;
    c->d_pin.release();
    c->d_pout.release();
    c->f_src.release();
    c->f_cnt.release();
    c->f_tile.release();
    c->f_rec.release();
    c->f_bound.release();
    c->r_bound.release();
    c->r_idx.release();
    c->r_cnt.release();
    c->r_sel.release();
    c->r_temp.release();
    c->r_cval.release();
    c->r_cval_s.release();
    c->r_cbeg.release();
    c->r_ckey.release();
    c->r_ckey_s.release();
    c->h_st.release();
    c->he_kind.release();
    c->he_temp.release();
    c->h_ring.release();
    DevBuf<int64_t>* h64[] = {&c->h_last, &c->h_tick, &c->h_mem, &c->he_t, &c->he_mem, &c->he_packed};
    for (auto* b : h64) b->release();
    DevBuf<int32_t>* h32[] = {&c->h_tests, &c->he_inv, &c->he_key, &c->he_idx0, &c->he_idx1,
                              &c->he_beg,  &c->he_end, &c->he_reg, &c->he_pad};
    for (auto* b : h32) b->release();
    if (c->ev_engine[0]) (void)hipEventDestroy(c->ev_engine[0]);
    if (c->ev_engine[1]) (void)hipEventDestroy(c->ev_engine[1]);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* owgs_last_error(const owgs_ctx* c) { return c ? c->err.c_str() : "null context"; }

// SCPB:512-551
int owgs_update_invokers(owgs_ctx* c, int32_t n, const int32_t* ids, const int64_t* user_memory_bytes,
                         const uint8_t* status) {
    if (!c || n < 0 || (n > 0 && (!ids || !user_memory_bytes || !status))) return OWGS_EINVAL;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    const int32_t old_size = (int32_t)c->ids.size();
    const int32_t new_size = n;
    bool large_next = false;
    int32_t managed = d2i(std::ceil((double)new_size * c->mf));
    if (managed < 1) managed = 1;
    int32_t blackboxes = d2i(std::floor((double)new_size * c->bf));
    if (blackboxes < 1) blackboxes = 1;
    if (managed > owgs_coprime_max() || blackboxes > owgs_coprime_max())
        return c->fail(OWGS_ERANGE, "pool larger than the step-size kernel's range");
    {  // validate before mutating: the state this update leads to must fit an engine geometry
        const int32_t slots = (old_size < new_size && n > c->n_slots) ? n : c->n_slots;
        bool identity = n <= slots;
        for (int32_t i = 0; identity && i < n; ++i) identity = ids[i] == i;
        // (a context already on the large-state engine stays there: its NestedSemaphore map lives in that layout;
        // slots never shrink, so a pool that left the chip cannot fit it again anyway)
        large_next = c->large || c->big_conc ||
                     engine_variant(slots, identity ? 0 : 1, n, std::min(managed, n), std::min(blackboxes, n)) < 0;
        if (large_next && !(identity && large_fits(n, std::min(managed, n), std::min(blackboxes, n))))
            return c->fail(OWGS_ERANGE, "invoker state exceeds every engine (owgs_limits; explicit pools on chip only)");
    }
    if (c->status_stale) {  // a device-only health update still in flight must land before the upload below
        HIPCHK(c, hipEventSynchronize(c->ev_status));
        c->status_stale = false;
    }
    c->ids.assign(ids, ids + n);
    c->mem.assign(user_memory_bytes, user_memory_bytes + n);
    c->status.assign(status, status + n);
    c->managed = managed;
    c->blackboxes = blackboxes;
    c->pool_override[0] = c->pool_override[1] = false;
    HIPCHK(c, upload(c->d_mem_bytes, user_memory_bytes, (size_t)n, c->stream));
    HIPCHK(c, upload(c->d_status, status, (size_t)n, c->stream));
    if (old_size != new_size) {
        // pairwiseCoprimeNumbersUntil(managed / blackboxes) on the device (owgs_state.hip), both pools in one launch
        const int32_t stride = std::max(managed, blackboxes);
        HIPCHK(c, c->d_steps.reserve((size_t)2 * stride));
        HIPCHK(c, c->d_cpx.reserve(4));
        int32_t xs[2] = {managed, blackboxes};
        HIPCHK(c, hipMemcpyAsync(c->d_cpx.p, xs, sizeof(xs), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, owgs_launch_coprime(c->d_cpx.p, 2, c->d_steps.p, stride, c->d_cpx.p + 2, c->stream));
        int32_t cnt[2];
        HIPCHK(c, hipMemcpyAsync(cnt, c->d_cpx.p + 2, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->steps_stride = stride;
        // host copies of the lists: introspection only (owgs_step_sizes); the prepare kernel reads d_steps
        c->msteps.resize((size_t)cnt[0]);
        c->bsteps.resize((size_t)cnt[1]);
        if (cnt[0]) HIPCHK(c, hipMemcpyAsync(c->msteps.data(), c->d_steps.p, (size_t)cnt[0] * 4, hipMemcpyDeviceToHost, c->stream));
        if (cnt[1])
            HIPCHK(c, hipMemcpyAsync(c->bsteps.data(), c->d_steps.p + stride, (size_t)cnt[1] * 4, hipMemcpyDeviceToHost,
                                     c->stream));
        if (old_size < new_size && n > c->n_slots) {
            // keep existing semaphores; append NestedSemaphore(getInvokerSlot(userMemory).toMB) for the new ones
            // (owgs_slots_kernel computes the tail in place)
            DevBuf<int32_t> nb;
            HIPCHK(c, nb.reserve((size_t)n));
            if (c->n_slots > 0)
                HIPCHK(c, hipMemcpyAsync(nb.p, c->d_permits.p, (size_t)c->n_slots * 4, hipMemcpyDeviceToDevice, c->stream));
            HIPCHK(c, owgs_launch_slots(c->d_mem_bytes.p, c->n_slots, n, c->cluster, c->cfg.min_memory_bytes, nb.p,
                                        c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            c->d_permits.release();
            c->d_permits = nb;
            nb.p = nullptr;
            c->n_slots = n;
        }
    }
    const bool was_large = c->large;
    c->large = large_next || c->big_conc;
    int rc = rebuild_pools(c);
    if (!rc && c->large && !was_large) rc = seq_migrate(c);
    if (!rc) rc = prepare_actions(c);
    if (!rc) HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!rc && !c->large) rc = lds_check(c);
    return rc;
}

// SCPB:561-584
int owgs_update_cluster(owgs_ctx* c, int32_t new_size) {
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    const int32_t actual = new_size > 1 ? new_size : 1;
    if (c->cluster == actual) return OWGS_OK;
    if (!c->large) {
        int rw = w_rebuild(c);  // in-flight concurrent activations of the discarded entries become watched pairs
        if (rw) return rw;
    } else if (c->q_cap > 0) {  // large-state engine: the map (with its empty entries) is discarded with the slots
        HIPCHK(c, hipMemsetAsync(c->q_map.p, 0, (size_t)c->q_cap * sizeof(uint4), c->stream));
        HIPCHK(c, hipMemsetAsync(c->q_filled.p, 0, 4, c->stream));
    }
    c->cluster = actual;
    const int32_t n = (int32_t)c->ids.size();
    HIPCHK(c, c->d_permits.reserve((size_t)n));
    HIPCHK(c, owgs_launch_slots(c->d_mem_bytes.p, 0, n, c->cluster, c->cfg.min_memory_bytes, c->d_permits.p,
                                c->stream));
    c->n_slots = n;
    int rc = c->large ? OWGS_OK : reset_ctab(c);
    if (!rc) rc = rebuild_pools(c);
    if (!rc) HIPCHK(c, hipStreamSynchronize(c->stream));
    return rc;
}

int owgs_register_actions(owgs_ctx* c, int32_t n, const char* ns_bytes, const int32_t* ns_off,
                          const char* path_bytes, const int32_t* path_off, const char* key_bytes,
                          const int32_t* key_off, const int32_t* mem_mb, const int32_t* max_conc,
                          const uint8_t* blackbox, int32_t* out_action, int32_t* out_hash) {
    if (c) ++c->res_cache_epoch;
    if (!c || n < 0) return OWGS_EINVAL;
    if (n == 0) return OWGS_OK;
    if (!ns_off || !path_off || !key_off || !mem_mb || !max_conc || !blackbox || !key_bytes || !out_action)
        return OWGS_EINVAL;
    for (int32_t i = 0; i < n; ++i) {
        // MemoryLimit/ConcurrencyLimit guarantee positive values (MemoryLimit.scala:68-69); the reference's
        // require(...) checks (FS:96, NS:85) would throw on anything else
        if (mem_mb[i] <= 0 || mem_mb[i] > OWGS_MAX_MEM_MB || max_conc[i] < 1)
            return c->fail(OWGS_EINVAL, "mem/maxConcurrent");
        if (ns_off[i + 1] < ns_off[i] || path_off[i + 1] < path_off[i] || key_off[i + 1] < key_off[i])
            return c->fail(OWGS_EINVAL, "offsets");
        // beyond the on-chip map's field: the large-state engine, which walks identity pools only
        if (max_conc[i] > OWGS_MAX_CONC && !c->big_conc && !c->ids.empty() && c->pool_mode != 0)
            return c->fail(OWGS_ERANGE, "maxConcurrent beyond 4095 needs identity pools");
    }
    // handles: released ones first, then new ids below OWGS_REC_NOACT
    if ((size_t)n > c->free_handles.size() + ((size_t)OWGS_REC_NOACT - c->a_mem.size()))
        return c->fail(OWGS_ERANGE, "too many live actions (release unused handles: owgs_release_actions)");
    // validate before mutating: one fqn@version has one set of limits (the action document is versioned)
    size_t fresh = 0;
    {
        std::unordered_map<std::string, std::pair<int32_t, int32_t>> seen;
        for (int32_t i = 0; i < n; ++i) {
            std::string k(key_bytes + key_off[i], (size_t)(key_off[i + 1] - key_off[i]));
            auto it = c->slot_ids.find(k);
            std::pair<int32_t, int32_t> lim{max_conc[i], mem_mb[i]};
            if (it != c->slot_ids.end()) {
                if (c->slot_maxc[it->second] != lim.first || c->slot_mem[it->second] != lim.second)
                    return c->fail(OWGS_EINVAL, "same fqn@version registered with different limits");
                continue;
            }
            auto sj = seen.find(k);
            if (sj == seen.end()) {
                seen.emplace(std::move(k), lim);
                ++fresh;
            } else if (sj->second != lim) {
                return c->fail(OWGS_EINVAL, "same fqn@version registered with different limits");
            }
        }
    }
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    // key ids: recycled ones, then new ones up to OWGS_MAX_SLOTKEYS; when they run out, recycle the keys no live
    // handle names and no map entry / watched pair holds any more
    auto key_room = [&]() { return c->free_slots.size() + ((size_t)OWGS_MAX_SLOTKEYS + 1 - c->slot_name.size()); };
    if (fresh > key_room()) {
        const int rr = reclaim_slots(c);
        if (rr) return rr;
        if (fresh > key_room()) return c->fail(OWGS_ERANGE, "too many live fqn@version keys");
    }
    c->cw_cache = 0;
    std::vector<int32_t> hid((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
        std::string k(key_bytes + key_off[i], (size_t)(key_off[i + 1] - key_off[i]));
        auto it = c->slot_ids.find(k);
        int32_t sid;
        if (it == c->slot_ids.end()) {
            if (!c->free_slots.empty()) {
                sid = c->free_slots.back();
                c->free_slots.pop_back();
                c->slot_name[sid] = k;
                c->slot_uses[sid] = 0;
                c->slot_maxc[sid] = max_conc[i];
                c->slot_mem[sid] = mem_mb[i];
            } else {
                sid = (int32_t)c->slot_name.size();
                c->slot_name.push_back(k);
                c->slot_uses.push_back(0);
                c->slot_maxc.push_back(max_conc[i]);
                c->slot_mem.push_back(mem_mb[i]);
            }
            c->slot_ids.emplace(std::move(k), sid);
        } else {
            sid = it->second;
        }
        c->slot_uses[sid]++;
        int32_t a;
        if (!c->free_handles.empty()) {
            a = c->free_handles.back();
            c->free_handles.pop_back();
        } else {
            a = (int32_t)c->a_mem.size();
            c->a_slot.push_back(0);
            c->a_mem.push_back(0);
            c->a_maxc.push_back(0);
            c->a_bb.push_back(0);
            c->a_hash.push_back(0);
            c->a_live.push_back(0);
        }
        c->a_slot[a] = sid;
        c->a_mem[a] = mem_mb[i];
        c->a_maxc[a] = max_conc[i];
        c->a_bb[a] = blackbox[i] ? 1 : 0;
        c->a_live[a] = 1;
        if (max_conc[i] > 1) c->any_conc = true;
        if (max_conc[i] > OWGS_MAX_CONC) c->big_conc = true;  // (checked above: identity pools)
        hid[i] = a;
        out_action[i] = a;
    }
    if (c->big_conc && !c->large) {  // beyond the on-chip map's field: move the slot state to the large-state engine
        c->large = true;
        const int rm = seq_migrate(c);
        if (rm) return rm;
    }
    const int32_t total = (int32_t)c->a_mem.size();
    // strings -> device, hash on the GPU
    DevBuf<char> dns, dpath;
    DevBuf<int32_t> dnso, dpo, dh;
    const size_t nsb = (size_t)ns_off[n], pb = (size_t)path_off[n];
    HIPCHK(c, upload(dns, ns_bytes, nsb, c->stream));
    HIPCHK(c, upload(dpath, path_bytes, pb, c->stream));
    HIPCHK(c, upload(dnso, ns_off, (size_t)n + 1, c->stream));
    HIPCHK(c, upload(dpo, path_off, (size_t)n + 1, c->stream));
    HIPCHK(c, dh.reserve((size_t)n));
    OwgsHashArgs ha{dns.p, dnso.p, dpath.p, dpo.p, n, 0, dh.p};
    HIPCHK(c, owgs_launch_hash(&ha, c->stream));
    std::vector<int32_t> h(n);
    HIPCHK(c, hipMemcpyAsync(h.data(), dh.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dns.release();
    dpath.release();
    dnso.release();
    dpo.release();
    dh.release();
    for (int32_t i = 0; i < n; ++i) {
        c->a_hash[hid[i]] = h[i];
        if (out_hash) out_hash[i] = h[i];
    }
    HIPCHK(c, upload(c->d_act_hash, c->a_hash.data(), (size_t)total, c->stream));
    HIPCHK(c, upload(c->d_act_slot, c->a_slot.data(), (size_t)total, c->stream));
    HIPCHK(c, upload(c->d_act_mem, c->a_mem.data(), (size_t)total, c->stream));
    HIPCHK(c, upload(c->d_act_maxc, c->a_maxc.data(), (size_t)total, c->stream));
    HIPCHK(c, upload(c->d_act_bb, c->a_bb.data(), (size_t)total, c->stream));
    // a walk cursor is exact for maxConcurrent==1 actions and for fqns invoked on a single walk; released
    // handles keep their last word (never read)
    c->a_cok.resize((size_t)total);
    for (int32_t a = 0; a < total; ++a)
        c->a_cok[a] = (c->a_live[a] && (c->a_maxc[a] == 1 || c->slot_uses[c->a_slot[a]] == 1)) ? 1 : 0;
    HIPCHK(c, upload(c->d_act_cok, c->a_cok.data(), (size_t)total, c->stream));
    int rc = prepare_actions(c);
    if (!rc) HIPCHK(c, hipStreamSynchronize(c->stream));
    return rc;
}

// The caller drops action handles (a cold action, a superseded fqn@version): no later call names them and none of
// their activations is still in flight.  Their ids, and the fqn@version keys no live handle names any more, are reused
// by later registrations -- the keys once nothing on the device holds them (reclaim_slots).
int owgs_release_actions(owgs_ctx* c, int32_t n, const int32_t* actions) {
    if (c) ++c->res_cache_epoch;
    if (!c || n < 0 || (n > 0 && !actions)) return OWGS_EINVAL;
    const int32_t na = (int32_t)c->a_mem.size();
    std::vector<uint8_t> seen;
    for (int32_t i = 0; i < n; ++i) {
        const int32_t a = actions[i];
        if (a < 0 || a >= na || !c->a_live[a]) return c->fail(OWGS_ENOENT, "unknown or released action");
        if (seen.empty()) seen.assign((size_t)na, 0);
        if (seen[a]++) return c->fail(OWGS_EINVAL, "action released twice in one call");
    }
    for (int32_t i = 0; i < n; ++i) {
        const int32_t a = actions[i], sid = c->a_slot[a];
        c->a_live[a] = 0;
        c->free_handles.push_back(a);
        if (--c->slot_uses[sid] == 0) c->pending_slots.push_back(sid);
    }
    if (n > 0) c->cw_cache = 0;
    return OWGS_OK;
}

int owgs_publish_batch(owgs_ctx* c, int32_t n, const int32_t* action, const uint64_t* seq, uint64_t seq_base,
                       int32_t* out_invoker, uint8_t* out_flags) {
    if (!c || n < 0 || (n > 0 && (!action || !out_invoker || !out_flags))) return OWGS_EINVAL;
    const CallTimer timer_(c);
    if (n == 0) return OWGS_OK;
    if (!registered(c, n, action)) return c->fail(OWGS_ENOENT, "unknown action");
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    if (c->large) {
        const int32_t ro[2] = {0, 0}, po[2] = {0, n};
        return seq_host_runs(c, 1, ro, nullptr, nullptr, nullptr, po, action, seq, seq_base, out_invoker, out_flags);
    }
    const int64_t off[2] = {0, n};
    HIPCHK(c, upload(c->d_off, off, 2, c->stream));
    HIPCHK(c, upload(c->d_a, action, (size_t)n, c->stream));
    if (seq) HIPCHK(c, upload(c->d_seq, (const u64*)seq, (size_t)n, c->stream));
    HIPCHK(c, c->d_out.reserve((size_t)n));
    HIPCHK(c, c->d_flags.reserve((size_t)n));
    OwgsEngineArgs A;
    base_args(c, A);
    A.seq_base = seq_base;
    A.seq = seq ? c->d_seq.p : nullptr;
    A.out_inv = c->d_out.p;
    A.out_flags = c->d_flags.p;
    int rc = run_prepass(c, A, 1, c->d_off.p, c->d_a.p, n, c->stream);
    if (!rc) rc = run_engine(c, A, c->stream);
    if (!rc) rc = w_update(c, n, c->d_a.p, c->d_out.p, c->d_flags.p, c->stream);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(out_invoker, c->d_out.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out_flags, c->d_flags.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return check_err_word(c);
}

// scratch of the release front end for n releases
static int release_scratch(owgs_ctx* c, OwgsReleaseArgs& R, int32_t n) {
    HIPCHK(c, c->r_bound.reserve((size_t)std::max(c->n_slots, 1)));
    HIPCHK(c, c->r_idx.reserve((size_t)std::max(n, 1)));
    HIPCHK(c, c->r_sel.reserve((size_t)std::max(n, 1)));
    HIPCHK(c, c->r_cnt.reserve(2));
    const size_t tb = owgs_release_scratch_bytes(std::max(n, 1));
    HIPCHK(c, c->r_temp.reserve(tb));
    R.bound = c->r_bound.p;
    R.risk = c->r_cnt.p + 1;
    R.sel_flag = c->r_sel.p;
    R.sel_idx = c->r_idx.p;
    R.sel_cnt = c->r_cnt.p;
    R.temp = c->r_temp.p;
    R.temp_bytes = tb;
    const size_t m = (size_t)std::max(n, 1);
    HIPCHK(c, c->r_ckey.reserve(m));
    HIPCHK(c, c->r_ckey_s.reserve(m));
    HIPCHK(c, c->r_cval.reserve(m));
    HIPCHK(c, c->r_cval_s.reserve(m));
    HIPCHK(c, c->r_cbeg.reserve(2 * OWGS_CTC));
    R.ckey = c->r_ckey.p;
    R.ckey_s = c->r_ckey_s.p;
    R.cval = c->r_cval.p;
    R.cval_s = c->r_cval_s.p;
    R.cbeg = c->r_cbeg.p;
    R.cend = c->r_cbeg.p + OWGS_CTC;
    return OWGS_OK;
}

// The exact release path (owgs_launch_release_seq: parallel front end, ordered kernel for overflow risk, watched pairs
// and entries counting at or below zero) for n releases already on the device.  Asynchronous on s.
static int release_chain(owgs_ctx* c, int32_t n, const int32_t* inv, const int32_t* mem, const int32_t* maxc,
                         const int32_t* slot, uint8_t* flags, hipStream_t s) {
    OwgsReleaseArgs R{};
    R.permits = c->d_permits.p;
    R.n_slots = c->n_slots;
    R.ct_keys = c->d_ct_keys.p;
    R.ct_vals = c->d_ct_vals.p;
    R.n = n;
    R.inv = inv;
    R.mem = mem;
    R.maxc = maxc;
    R.slot = slot;
    R.flags = flags;
    R.err = c->d_err.p;
    int rs = release_scratch(c, R, n);
    if (!rs && c->w_cap > 0) {  // room for the empty entries releases of watched pairs meet
        rs = ensure_ovf(c, n, s);
        ovf_add(c, n);
    }
    if (rs) return rs;
    R.ovf = ovf_args(c);
    R.w = watch_args(c);
    HIPCHK(c, owgs_launch_release_seq(&R, s));
    return OWGS_OK;
}

int owgs_release_batch(owgs_ctx* c, int32_t n, const int32_t* invoker, const int32_t* action, uint8_t* out_flags) {
    const CallTimer timer_(c);
    if (!c || n < 0 || (n > 0 && (!invoker || !action))) return OWGS_EINVAL;
    if (n == 0) return OWGS_OK;
    if (!registered(c, n, action)) return c->fail(OWGS_ENOENT, "unknown action");
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    if (c->large) {
        const int32_t ro[2] = {0, n}, po[2] = {0, 0};
        std::vector<uint8_t> fl((size_t)n);
        const int rc = seq_host_runs(c, 1, ro, invoker, action, fl.data(), po, nullptr, nullptr, 0, nullptr, nullptr);
        if (out_flags) memcpy(out_flags, fl.data(), (size_t)n);
        return rc;
    }
    std::vector<int32_t> mem(n), mc(n), sl(n);
    for (int32_t i = 0; i < n; ++i) {
        mem[i] = c->a_mem[action[i]];
        mc[i] = c->a_maxc[action[i]];
        sl[i] = c->a_slot[action[i]];
    }
    HIPCHK(c, upload(c->d_a, invoker, (size_t)n, c->stream));
    HIPCHK(c, upload(c->d_b, mem.data(), (size_t)n, c->stream));
    HIPCHK(c, upload(c->d_c, mc.data(), (size_t)n, c->stream));
    HIPCHK(c, upload(c->d_d, sl.data(), (size_t)n, c->stream));
    HIPCHK(c, c->d_rflags.reserve((size_t)n));
    int rs = release_chain(c, n, c->d_a.p, c->d_b.p, c->d_c.p, c->d_d.p, c->d_rflags.p, c->stream);
    if (rs) return rs;
    if (out_flags)
        HIPCHK(c, hipMemcpyAsync(out_flags, c->d_rflags.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    rs = w_refresh(c, c->stream);
    return rs ? rs : check_err_word(c);
}

int owgs_schedule_walks(owgs_ctx* c, int32_t n, const uint8_t* pool, const int32_t* index, const int32_t* step,
                        const int32_t* mem_mb, const int32_t* max_conc, const int32_t* key, const uint64_t* seq,
                        int32_t* out_invoker, uint8_t* out_flags) {
    if (!c || n < 0 || (n > 0 && (!pool || !index || !step || !mem_mb || !max_conc || !key || !out_invoker || !out_flags)))
        return OWGS_EINVAL;
    OWGS_NOT_LARGE(c);
    if (n == 0) return OWGS_OK;
    std::vector<uint2> xm(n);
    for (int32_t i = 0; i < n; ++i) {
        if (mem_mb[i] <= 0 || mem_mb[i] > OWGS_MAX_MEM_MB || max_conc[i] < 1 || max_conc[i] > OWGS_MAX_CONC ||
            step[i] < 0 || step[i] > (1 << 30) || key[i] < 0 || key[i] > OWGS_MAX_SLOTKEYS)
            return c->fail(OWGS_EINVAL, "mem/maxConcurrent/step");
        const int p = pool[i] ? 1 : 0;
        const int32_t np = p ? c->nb : c->nm;
        uint32_t y = (uint32_t)mem_mb[i] | ((uint32_t)max_conc[i] << OWGS_AM_MAXC_SHIFT);
        uint32_t x = p ? OWGS_AM_POOL : 0u;
        if (np == 0) {
            y |= OWGS_AM_EMPTY;
        } else if (index[i] < 0 || index[i] >= np) {
            y |= OWGS_AM_THROW;
        } else {
            x |= (uint32_t)index[i] | ((uint32_t)(step[i] % np) << 15);  // same walk (Java %)
        }
        xm[i] = make_uint2(x, y);  // no cursor: explicit walks are independent
    }
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    const int64_t off[2] = {0, n};
    HIPCHK(c, upload(c->d_off, off, 2, c->stream));
    HIPCHK(c, upload(c->d_xmeta, xm.data(), (size_t)n, c->stream));
    HIPCHK(c, upload(c->d_xslot, key, (size_t)n, c->stream));
    if (seq) HIPCHK(c, upload(c->d_seq, (const u64*)seq, (size_t)n, c->stream));
    HIPCHK(c, c->d_out.reserve((size_t)n));
    HIPCHK(c, c->d_flags.reserve((size_t)n));
    OwgsEngineArgs A;
    base_args(c, A);
    A.feat = OWGS_F_ALL;  // explicit walks carry their own limits
    A.seq = seq ? c->d_seq.p : nullptr;
    A.out_inv = c->d_out.p;
    A.out_flags = c->d_flags.p;
    int rc = run_prepass(c, A, 1, c->d_off.p, nullptr, n, c->stream);
    if (!rc) rc = run_engine(c, A, c->stream);
    if (!rc) rc = w_update(c, n, nullptr, c->d_out.p, c->d_flags.p, c->stream);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(out_invoker, c->d_out.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out_flags, c->d_flags.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return check_err_word(c);
}

int owgs_set_slots(owgs_ctx* c, int32_t n, const int32_t* permits) {
    if (!c || n < 0 || (n > 0 && !permits)) return OWGS_EINVAL;
    OWGS_NOT_LARGE(c);
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    int rw = w_rebuild(c);
    if (rw) return rw;
    HIPCHK(c, upload(c->d_permits, permits, (size_t)n, c->stream));
    c->n_slots = n;
    int rc = reset_ctab(c);
    if (!rc) rc = rebuild_pools(c);
    if (!rc) HIPCHK(c, hipStreamSynchronize(c->stream));
    return rc;
}

int owgs_set_pool(owgs_ctx* c, int32_t pool, int32_t n, const int32_t* ids, const uint8_t* status) {
    if (!c || (pool != 0 && pool != 1) || n < 0 || (n > 0 && (!ids || !status))) return OWGS_EINVAL;
    OWGS_NOT_LARGE(c);
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    c->pool_override[pool] = true;
    c->ov_ids[pool].assign(ids, ids + n);
    c->ov_status[pool].assign(status, status + n);
    int rc = rebuild_pools(c);
    if (!rc) rc = prepare_actions(c);
    if (!rc) HIPCHK(c, hipStreamSynchronize(c->stream));
    return rc;
}

int owgs_read_permits(owgs_ctx* c, int32_t* out, int32_t cap, int32_t* n_slots) {
    if (!c) return OWGS_EINVAL;
    if (n_slots) *n_slots = c->n_slots;
    if (!out || cap <= 0 || c->n_slots == 0) return OWGS_OK;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, c->d_permits.p, (size_t)std::min(cap, c->n_slots) * 4, hipMemcpyDeviceToHost));
    return OWGS_OK;
}

int owgs_read_concurrent(owgs_ctx* c, int32_t invoker, int32_t key, int32_t* permits, int32_t* op_count) {
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    if (c->large) {  // the large-state engine's map (it holds the reference's empty entries too)
        HIPCHK(c, c->q_look.reserve(4));
        if (c->q_cap <= 0) return 0;
        OwgsSeqArgs S = seq_args(c);
        HIPCHK(c, owgs_launch_seq_lookup(&S, invoker, key, c->q_look.p, c->stream));
        int32_t v[3];
        HIPCHK(c, hipMemcpyAsync(v, c->q_look.p, sizeof(v), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (!v[0]) return 0;
        if (permits) *permits = v[1];
        if (op_count) *op_count = v[2];
        return 1;
    }
    DevBuf<int32_t> di, dk;
    DevBuf<int2> dv;
    HIPCHK(c, upload(di, &invoker, 1, c->stream));
    HIPCHK(c, upload(dk, &key, 1, c->stream));
    HIPCHK(c, dv.reserve(1));
    OwgsLookupArgs la{c->d_ct_keys.p, c->d_ct_vals.p, ovf_args(c), di.p, dk.p, 1, dv.p};
    HIPCHK(c, owgs_launch_lookup(&la, c->stream));
    int2 v;
    HIPCHK(c, hipMemcpyAsync(&v, dv.p, sizeof(int2), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    di.release();
    dk.release();
    dv.release();
    if (v.x < 0) return 0;  // absent (NestedSemaphore.concurrentState has no entry); present entries may count <= 0
    if (permits) *permits = v.x;
    if (op_count) *op_count = v.y;
    return 1;
}

int owgs_map_fill(owgs_ctx* c, int32_t* primary_live, int32_t* primary_deleted, int32_t* overflow_entries,
                  int32_t* overflow_cap) {
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<uint32_t> k(OWGS_CTC);
    int32_t oc = 0;
    if (c->d_ct_keys.p) HIPCHK(c, hipMemcpy(k.data(), c->d_ct_keys.p, OWGS_CTC * 4, hipMemcpyDeviceToHost));
    if (c->ovf_cap > 0 && c->d_ovf_cnt.p) HIPCHK(c, hipMemcpy(&oc, c->d_ovf_cnt.p, 4, hipMemcpyDeviceToHost));
    int32_t live = 0, del = 0;
    for (uint32_t x : k) {
        live += x != 0u && x != OWGS_CT_TOMB;
        del += x == OWGS_CT_TOMB;
    }
    if (primary_live) *primary_live = c->d_ct_keys.p ? live : 0;
    if (primary_deleted) *primary_deleted = c->d_ct_keys.p ? del : 0;
    if (overflow_entries) *overflow_entries = oc;
    if (overflow_cap) *overflow_cap = c->ovf_cap;
    return OWGS_OK;
}

int owgs_key_id(owgs_ctx* c, int32_t action) {
    if (!c || action < 0 || action >= (int32_t)c->a_slot.size() || !c->a_live[action]) return OWGS_ENOENT;
    return c->a_slot[action];
}

int owgs_state_info(owgs_ctx* c, int32_t* n_invokers, int32_t* managed, int32_t* blackbox, int32_t* cluster_size) {
    if (!c) return OWGS_EINVAL;
    if (n_invokers) *n_invokers = (int32_t)c->ids.size();
    if (managed) *managed = c->nm;
    if (blackbox) *blackbox = c->nb;
    if (cluster_size) *cluster_size = c->cluster;
    return OWGS_OK;
}

int owgs_step_sizes(owgs_ctx* c, int32_t pool, int32_t* out, int32_t cap, int32_t* n) {
    if (!c || (pool != 0 && pool != 1)) return OWGS_EINVAL;
    const std::vector<int32_t>& v = pool ? c->bsteps : c->msteps;
    if (n) *n = (int32_t)v.size();
    for (int32_t i = 0; out && i < cap && i < (int32_t)v.size(); ++i) out[i] = v[i];
    return OWGS_OK;
}

int owgs_pairwise_coprime(owgs_ctx* c, int32_t x, int32_t* out, int32_t cap, int32_t* n) {
    if (!c || cap < 0) return OWGS_EINVAL;
    if (x > owgs_coprime_max()) return c->fail(OWGS_ERANGE, "x beyond the step-size kernel's range");
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    DevBuf<int32_t> d;
    HIPCHK(c, d.reserve((size_t)std::max(x, 0) + 2));
    HIPCHK(c, hipMemcpyAsync(d.p, &x, 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, owgs_launch_coprime(d.p, 1, d.p + 2, std::max(x, 1), d.p + 1, c->stream));
    int32_t cnt = 0;
    HIPCHK(c, hipMemcpyAsync(&cnt, d.p + 1, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (out && cap > 0 && cnt > 0)
        HIPCHK(c, hipMemcpy(out, d.p + 2, (size_t)std::min(cap, cnt) * 4, hipMemcpyDeviceToHost));
    if (n) *n = cnt;
    d.release();
    return OWGS_OK;
}

static int replay_begin(owgs_ctx* c, int32_t n_batches, const int64_t* acq_off, const int32_t* act,
                        int64_t n_activations, const int64_t* rel_off, const int64_t* rel_aid, int64_t n_releases,
                        uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags, uint8_t* rel_flags,
                        hipStream_t hs, OwgsEngineArgs& A, bool launch);

// Replay in watch mode (watched pairs exist): batch by batch, so that the Z marks of a batch's publishes are in place
// before the next batch's releases -- releases through the ordered release kernels, publishes through one engine
// launch per batch, then the watch update.  Reads the batch offsets back once (synchronous).
static int replay_watch(owgs_ctx* c, int32_t nb, const int64_t* acq_off, const int32_t* act, int64_t n_act,
                        const int64_t* rel_off, const int64_t* rel_aid, int64_t n_rel, uint64_t seq_base,
                        int32_t* out_inv, uint8_t* out_flags, uint8_t* rel_flags, hipStream_t hs) {
    (void)n_act;
    (void)n_rel;
    std::vector<int64_t> ao((size_t)nb + 1), ro((size_t)nb + 1, 0);
    HIPCHK(c, hipMemcpyAsync(ao.data(), acq_off, ao.size() * 8, hipMemcpyDeviceToHost, hs));
    if (rel_off) HIPCHK(c, hipMemcpyAsync(ro.data(), rel_off, ro.size() * 8, hipMemcpyDeviceToHost, hs));
    HIPCHK(c, hipStreamSynchronize(hs));
    std::vector<int64_t> offs((size_t)2 * nb);
    int64_t max_r = 1;
    for (int32_t b = 0; b < nb; ++b) {
        offs[2 * b] = 0;
        offs[2 * b + 1] = ao[b + 1] - ao[b];
        max_r = std::max(max_r, ro[b + 1] - ro[b]);
    }
    HIPCHK(c, upload(c->w_off, offs.data(), offs.size(), hs));
    HIPCHK(c, c->w_rel.reserve((size_t)(4 * max_r)));
    if (!rel_flags) HIPCHK(c, c->w_rfl.reserve((size_t)max_r));
    for (int32_t b = 0; b < nb; ++b) {
        const int64_t nr = ro[b + 1] - ro[b], na = ao[b + 1] - ao[b];
        if (nr > 0) {  // releaseInvoker of the batch's completions (SCPB:327-331), in stream order
            int32_t* q = c->w_rel.p;
            HIPCHK(c, owgs_launch_w_relgather(rel_aid + ro[b], (int32_t)nr, out_inv, act, c->d_act_mem.p,
                                              c->d_act_maxc.p, c->d_act_slot.p, q, q + max_r, q + 2 * max_r,
                                              q + 3 * max_r, hs));
            int rs = release_chain(c, (int32_t)nr, q, q + max_r, q + 2 * max_r, q + 3 * max_r,
                                   rel_flags ? rel_flags + ro[b] : c->w_rfl.p, hs);
            if (rs) return rs;
        }
        if (na > 0) {  // the batch's publishes (SCPB:257-290), then the watch marks of their walks
            OwgsEngineArgs A;
            base_args(c, A);
            A.seq_base = seq_base + (uint64_t)ao[b];
            A.out_inv = out_inv + ao[b];
            A.out_flags = out_flags + ao[b];
            int rc = run_prepass(c, A, 1, c->w_off.p + 2 * b, act + ao[b], na, hs);
            if (!rc) rc = run_engine(c, A, hs);
            if (!rc) rc = w_update(c, (int32_t)na, act + ao[b], out_inv + ao[b], out_flags + ao[b], hs);
            if (rc) return rc;
        }
    }
    return w_refresh(c, hs);
}

static bool spec_replay_eligible(const owgs_ctx* c);
static int spec_replay(owgs_ctx* c, int32_t nb, const int64_t* acq_off, const int32_t* act, int64_t n_act,
                       const int64_t* rel_off, const int64_t* rel_aid, int64_t n_rel, uint64_t seq_base,
                       int32_t* out_inv, uint8_t* out_flags, uint8_t* rel_flags, hipStream_t hs, int64_t aid_end);

// One batch of a device-resident stream replayed batch by batch (state updates such as a health change in between):
// releases rel_aid[r_beg, r_end) of activations decided by earlier calls (invoker in out_invoker), then the publishes
// act[a_beg, a_end).  The releases are staged as engine records from the earlier decisions, so the batch is one
// engine launch (owgs_fused.hip span mode); with watched pairs: the exact release kernels + the watch update.
static int replay_device_span_impl(owgs_ctx* c, int64_t a_beg, int64_t a_end, int64_t r_beg, int64_t r_end, const int32_t* act,
                            const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags,
                            uint8_t* rel_flags, void* stream) {
    if (!c || a_beg < 0 || a_end < a_beg || r_beg < 0 || r_end < r_beg || !act || !out_invoker || !out_flags ||
        (r_end > r_beg && !rel_aid) || a_end - a_beg >= ((int64_t)1 << 31) || r_end - r_beg >= ((int64_t)1 << 31))
        return OWGS_EINVAL;
    if (c->a_mem.empty()) return c->fail(OWGS_ENOENT, "no actions registered");
    const int64_t na = a_end - a_beg, nr = r_end - r_beg;
    if (na == 0 && nr == 0) return OWGS_OK;
    OWGS_ENTER(c);
    hipStream_t hs = stream ? (hipStream_t)stream : c->stream;
    if (c->large) {  // one run: the batch's releases, then its publishes (whole-stream indices)
        const int64_t offs[4] = {r_beg, r_end, a_beg, a_end};
        HIPCHK(c, upload(c->g_off, offs, 4, hs));
        return seq_device_runs(c, 1, c->g_off.p, c->g_off.p + 2, act, rel_aid, seq_base, out_invoker, out_flags,
                               rel_flags, hs);
    }
    HIPCHK(c, c->w_rfl.reserve((size_t)std::max<int64_t>(nr, 1)));
    uint8_t* rf = rel_flags ? rel_flags + r_beg : c->w_rfl.p;
    if (c->w_cap > 0) {  // watched pairs: ordered release kernels, one engine launch, the watch update
        if (nr > 0) {
            HIPCHK(c, c->w_rel.reserve((size_t)(4 * nr)));
            int32_t* q = c->w_rel.p;
            HIPCHK(c, owgs_launch_w_relgather(rel_aid + r_beg, (int32_t)nr, out_invoker, act, c->d_act_mem.p,
                                              c->d_act_maxc.p, c->d_act_slot.p, q, q + nr, q + 2 * nr, q + 3 * nr, hs));
            int rs = release_chain(c, (int32_t)nr, q, q + nr, q + 2 * nr, q + 3 * nr, rf, hs);
            if (rs) return rs;
        }
        if (na > 0) {
            const int64_t offs[2] = {0, na};
            HIPCHK(c, upload(c->w_off, offs, 2, hs));
            OwgsEngineArgs A;
            base_args(c, A);
            A.seq_base = seq_base + (uint64_t)a_beg;
            A.out_inv = out_invoker + a_beg;
            A.out_flags = out_flags + a_beg;
            int rc = run_prepass(c, A, 1, c->w_off.p, act + a_beg, na, hs);
            if (!rc) rc = run_engine(c, A, hs);
            if (!rc) rc = w_update(c, (int32_t)na, act + a_beg, out_invoker + a_beg, out_flags + a_beg, hs);
            if (rc) return rc;
        }
        return w_refresh(c, hs);
    }
    if (spec_replay_eligible(c)) {  // one batch through the resident engine's stream mode
        const int64_t offs[4] = {a_beg, a_end, r_beg, r_end};
        HIPCHK(c, upload(c->w_off, offs, 4, hs));
        return spec_replay(c, 1, c->w_off.p, act, na, nr > 0 ? c->w_off.p + 2 : nullptr, rel_aid, nr, seq_base,
                           out_invoker, out_flags, rel_flags, hs, a_beg);
    }
    c->spec_last = false;
    HIPCHK(c, c->f_rec.reserve((size_t)nr + 2));
    HIPCHK(c, c->f_src.reserve((size_t)nr + 1));
    HIPCHK(c, c->f_cnt.reserve(2));
    HIPCHK(c, c->w_off.reserve(4));
    OwgsStageArgs g{};
    g.n_runs = 1;
    g.rel_off = nullptr;  // span mode
    g.rel_aid = rel_aid ? rel_aid + r_beg : nullptr;
    g.dec_inv = out_invoker;
    g.dec_act = act;
    g.span_nrel = nr;
    g.span_npub = na;
    g.span_off = c->w_off.p;
    g.act_mem = c->d_act_mem.p;
    g.act_maxc = c->d_act_maxc.p;
    g.act_slot = c->d_act_slot.p;
    g.n_slots = c->n_slots;
    g.rel_rec = c->f_rec.p;
    g.rel_src = c->f_src.p;
    g.relcnt = c->f_cnt.p;
    g.rel_flags = rf;
    HIPCHK(c, c->f_tile.reserve((size_t)(nr / OWGS_STAGE_TILE + 1)));
    g.tile_cnt = c->f_tile.p;
    HIPCHK(c, owgs_launch_stage_releases(&g, hs));
    OwgsEngineArgs A;
    base_args(c, A);
    A.seq_base = seq_base + (uint64_t)a_beg;
    A.out_inv = out_invoker + a_beg;
    A.out_flags = out_flags + a_beg;
    int rc = run_prepass(c, A, 1, c->w_off.p, act + a_beg, na, hs);
    if (!rc && nr > 0) {
        A.rel_off = c->w_off.p + 2;
        A.relcnt = c->f_cnt.p;
        A.rel_rec = c->f_rec.p;
        A.rel_src = c->f_src.p;
        A.rel_flags = rf;
    }
    if (!rc) rc = run_engine(c, A, hs);
    return rc;
}

int owgs_replay_device_span(owgs_ctx* c, int64_t a_beg, int64_t a_end, int64_t r_beg, int64_t r_end, const int32_t* act,
                            const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags,
                            uint8_t* rel_flags, void* stream) {
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    hipStream_t hs_ = stream ? (hipStream_t)stream : c->stream;
    int rc = order_on(c, hs_);
    if (!rc) rc = replay_device_span_impl(c, a_beg, a_end, r_beg, r_end, act, rel_aid, seq_base, out_invoker, out_flags, rel_flags, stream);
    const int rt = tail_mark(c, hs_);  // (also after a failure: whatever was enqueued stays ordered)
    return rc ? rc : rt;
}

// owgs_replay_device through the resident engine in stream mode (owgs_resident.hip): one workgroup loads the state,
// replays every batch -- its releases, then its publishes, in pieces the staging area holds -- with one wave deciding
// (speculative walks, in-order validation) and writes the state back.  Identity pools, no watched pairs.
static bool spec_replay_eligible(const owgs_ctx* c) {
    if (env_opts().spec_replay <= 0 || env_opts().res_spec <= 0 || c->pool_mode != 0 || c->w_cap > 0) return false;
    if (c->n_slots > OWGS_MAX_SLOTS_CT || c->n_ids > c->n_slots || c->nm > (int32_t)OWGS_AM_POS_MASK ||
        c->nb > (int32_t)OWGS_AM_POS_MASK || c->a_mem.empty())
        return false;
    return res_stage_bytes(c) >= 8192;
}

// (n_act: the call's activations; aid_end: the end of the activation index range the stream arrays cover)
static int spec_replay(owgs_ctx* c, int32_t nb, const int64_t* acq_off, const int32_t* act, int64_t n_act,
                       const int64_t* rel_off, const int64_t* rel_aid, int64_t n_rel, uint64_t seq_base,
                       int32_t* out_inv, uint8_t* out_flags, uint8_t* rel_flags, hipStream_t hs, int64_t aid_end) {
    if (c->any_conc) {
        const int rc = ensure_ovf(c, (int32_t)std::min<int64_t>(n_act, INT32_MAX), hs);
        if (rc) return rc;
        ovf_add(c, (int32_t)std::min<int64_t>(n_act, INT32_MAX));
    }
    HIPCHK(c, c->d_ct_tmp.reserve((size_t)2 * OWGS_CTC));
    const size_t na = std::max<size_t>(c->a_mem.size(), 1);
    // walk cursors: generations above every stored one; each release piece may start a new generation
    if (c->d_res_cur.n < na || (uint64_t)c->res_gen_seen + (uint64_t)n_rel + 2 >= 0xFFFFFF00ull) {
        HIPCHK(c, c->d_res_cur.reserve(std::max(na + na / 2, c->d_res_cur.n)));
        HIPCHK(c, hipMemsetAsync(c->d_res_cur.p, 0, c->d_res_cur.n * sizeof(uint2), hs));
        c->res_gen_seen = 0;
    }
    HIPCHK(c, c->d_spec_stats.reserve(OWGS_RES_NPROF));
    HIPCHK(c, hipMemsetAsync(c->d_spec_stats.p, 0, OWGS_RES_NPROF * sizeof(unsigned long long), hs));
    OwgsResArgs a{};
    a.permits = c->d_permits.p;
    a.n_slots = c->n_slots;
    a.usable = c->d_usable.p;
    a.n_ids = c->n_ids;
    a.nm = c->nm;
    a.nb = c->nb;
    a.ct_keys = c->d_ct_keys.p;
    a.ct_vals = c->d_ct_vals.p;
    a.ct_tmp = c->d_ct_tmp.p;
    a.ovf = ovf_args(c);
    a.act_meta = c->d_act_meta.p;
    a.act_slot = c->d_act_slot.p;
    a.n_actions = (int32_t)c->a_mem.size();
    a.rng_seed = c->cfg.rng_seed;
    a.err = c->d_err.p;
    a.stage_bytes = (int32_t)res_stage_bytes(c);
    a.cur = c->d_res_cur.p;
    a.gen_base = ++c->res_gen_seen;
    c->res_gen_seen += (uint32_t)n_rel + 1;
    a.spec = std::max(0, env_opts().res_spec);
    a.cspec = std::max(0, env_opts().res_cspec);
    a.cspec_pre = std::max(0, env_opts().res_cspec_pre);
    a.hsplit = std::max(0, std::min(3, env_opts().res_split));
    a.prespec = env_opts().res_pre;
    a.smode = 1;
    a.s_nb = nb;
    a.s_nact = aid_end;
    a.s_acq_off = acq_off;
    a.s_act = act;
    a.s_rel_off = n_rel > 0 ? rel_off : nullptr;
    a.s_rel_aid = rel_aid;
    a.s_seq_base = seq_base;
    a.s_out_inv = out_inv;
    a.s_out_fl = out_flags;
    a.s_rel_fl = rel_flags;
    a.s_stats = c->d_spec_stats.p;
    if (nb > 1 || aid_end == n_act) {  // a whole stream: every release names a distinct activation (spans: each alone)
        const size_t words = (size_t)(aid_end + 31) / 32 + 1;
        HIPCHK(c, c->d_claim.reserve(words));
        HIPCHK(c, hipMemsetAsync(c->d_claim.p, 0, words * sizeof(uint32_t), hs));
        a.s_claim = c->d_claim.p;
    }
    if (!c->ev_engine[0]) {
        HIPCHK(c, hipEventCreate(&c->ev_engine[0]));
        HIPCHK(c, hipEventCreate(&c->ev_engine[1]));
    }
    const size_t lds = owgs_resident_image_bytes(c->n_slots, c->n_ids) + (size_t)a.stage_bytes;
    HIPCHK(c, hipEventRecord(c->ev_engine[0], hs));
    HIPCHK(c, owgs_launch_resident(&a, lds, hs));
    HIPCHK(c, hipEventRecord(c->ev_engine[1], hs));
    c->ev_engine_valid = true;
    c->spec_last = true;
    return OWGS_OK;
}

static int replay_device_impl(owgs_ctx* c, int32_t n_batches, const int64_t* acq_off, const int32_t* act,
                       int64_t n_activations, const int64_t* rel_off, const int64_t* rel_aid, int64_t n_releases,
                       uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags, uint8_t* rel_flags, void* stream) {
    if (!c) return OWGS_EINVAL;
    hipStream_t hs = stream ? (hipStream_t)stream : c->stream;
    if (n_batches > 0 && c->large) {
        if (!acq_off || !act || !out_invoker || !out_flags || n_activations < 0 || n_releases < 0 ||
            (n_releases > 0 && (!rel_off || !rel_aid)))
            return OWGS_EINVAL;
        if (c->a_mem.empty()) return c->fail(OWGS_ENOENT, "no actions registered");
        const int64_t* ro = rel_off;
        if (!ro) {  // no releases: zero offsets
            std::vector<int64_t> z((size_t)n_batches + 1, 0);
            HIPCHK(c, upload(c->g_off, z.data(), z.size(), hs));
            ro = c->g_off.p;
        }
        return seq_device_runs(c, n_batches, ro, acq_off, act, rel_aid, seq_base, out_invoker, out_flags, rel_flags, hs);
    }
    if (n_batches > 0 && spec_replay_eligible(c)) {
        if (!acq_off || !act || !out_invoker || !out_flags || n_activations < 0 || n_activations >= ((int64_t)1 << 31) ||
            n_releases < 0 || (n_releases > 0 && (!rel_off || !rel_aid)))
            return OWGS_EINVAL;
        (void)hipSetDevice(c->cfg.device);
        return spec_replay(c, n_batches, acq_off, act, n_activations, rel_off, rel_aid, n_releases, seq_base,
                           out_invoker, out_flags, rel_flags, hs, n_activations);
    }
    c->spec_last = false;
    if (c->w_cap > 0 && n_batches > 0) {
        if (!acq_off || !act || !out_invoker || !out_flags || n_activations < 0 || n_releases < 0 ||
            (n_releases > 0 && (!rel_off || !rel_aid)))
            return OWGS_EINVAL;
        if (c->a_mem.empty()) return c->fail(OWGS_ENOENT, "no actions registered");
        (void)hipSetDevice(c->cfg.device);
        return replay_watch(c, n_batches, acq_off, act, n_activations, rel_off, rel_aid, n_releases, seq_base,
                            out_invoker, out_flags, rel_flags, hs);
    }
    OwgsEngineArgs A;
    int rc = replay_begin(c, n_batches, acq_off, act, n_activations, rel_off, rel_aid, n_releases, seq_base,
                          out_invoker, out_flags, rel_flags, hs, A, true);
    if (rc || n_batches == 0) return rc;
    if (rel_off && rel_flags) HIPCHK(c, owgs_launch_relflags(rel_aid, n_releases, out_invoker, rel_flags, hs));
    return OWGS_OK;
}

int owgs_replay_device(owgs_ctx* c, int32_t n_batches, const int64_t* acq_off, const int32_t* act,
                       int64_t n_activations, const int64_t* rel_off, const int64_t* rel_aid, int64_t n_releases,
                       uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags, uint8_t* rel_flags, void* stream) {
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    hipStream_t hs_ = stream ? (hipStream_t)stream : c->stream;
    int rc = order_on(c, hs_);
    if (!rc) rc = replay_device_impl(c, n_batches, acq_off, act, n_activations, rel_off, rel_aid, n_releases, seq_base, out_invoker, out_flags, rel_flags, stream);
    const int rt = tail_mark(c, hs_);  // (also after a failure: whatever was enqueued stays ordered)
    return rc ? rc : rt;
}

static int update_health_device_impl(owgs_ctx* c, int32_t n, const uint8_t* status_dev, void* stream);

// owgs_replay_device_group: batches [0, n) of the caller's host offsets in one engine launch, health row b applied by
// the engine before batch b (identity pools, no watched pairs); otherwise health + span per batch
static int replay_device_group_impl(owgs_ctx* c, int32_t nb, const int64_t* acq_off, const int64_t* rel_off,
                                    const int32_t* act, const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker,
                                    uint8_t* out_flags, uint8_t* rel_flags, const uint8_t* status_dev,
                                    int64_t status_stride, int32_t n_status, void* stream) {
    if (nb <= 0 || !acq_off || !rel_off || !act || !out_invoker || !out_flags) return OWGS_EINVAL;
    for (int32_t b = 0; b < nb; ++b)
        if (acq_off[b + 1] < acq_off[b] || rel_off[b + 1] < rel_off[b]) return c->fail(OWGS_EINVAL, "offsets");
    if (acq_off[0] < 0 || rel_off[0] < 0 || acq_off[nb] >= ((int64_t)1 << 31)) return c->fail(OWGS_EINVAL, "offsets");
    if (rel_off[nb] > rel_off[0] && !rel_aid) return OWGS_EINVAL;
    if (status_dev && (n_status <= 0 || status_stride < n_status)) return c->fail(OWGS_EINVAL, "health rows");
    if (c->a_mem.empty()) return c->fail(OWGS_ENOENT, "no actions registered");
    if (c->large || c->w_cap > 0 || c->pool_mode != 0 || spec_replay_eligible(c) ||
        (status_dev && n_status != c->n_ids)) {
        for (int32_t b = 0; b < nb; ++b) {  // the batch-by-batch sequence the call stands for
            int rc = status_dev ? update_health_device_impl(c, n_status, status_dev + (int64_t)b * status_stride, stream)
                                : OWGS_OK;
            if (!rc)
                rc = replay_device_span_impl(c, acq_off[b], acq_off[b + 1], rel_off[b], rel_off[b + 1], act, rel_aid,
                                             seq_base, out_invoker, out_flags, rel_flags, stream);
            if (rc) return rc;
        }
        return OWGS_OK;
    }
    hipStream_t hs = stream ? (hipStream_t)stream : c->stream;
    const int64_t a0 = acq_off[0], r0 = rel_off[0], n_rel = rel_off[nb] - r0;
    std::vector<int64_t> offs((size_t)2 * (nb + 1));
    for (int32_t b = 0; b <= nb; ++b) {
        offs[b] = acq_off[b];                      // absolute: the engine indexes the stream's arrays
        offs[nb + 1 + b] = rel_off[b] - r0;        // relative to the group's first release
    }
    HIPCHK(c, upload(c->g_off, offs.data(), offs.size(), hs));
    if (status_dev) {
        const int32_t words = (c->n_ids + 31) / 32;
        HIPCHK(c, c->d_hwords.reserve((size_t)nb * std::max(words, 1)));
        HIPCHK(c, owgs_launch_usable_rows(status_dev, status_stride, n_status, nb, c->d_hwords.p, words, hs));
        c->grp_hwords = c->d_hwords.p;
        c->grp_hstride = words;
    }
    c->grp_a0 = a0;
    OwgsEngineArgs A;
    int rc = replay_begin(c, nb, c->g_off.p, act, acq_off[nb], n_rel > 0 ? c->g_off.p + nb + 1 : nullptr,
                          n_rel > 0 ? rel_aid + r0 : nullptr, n_rel, seq_base, out_invoker, out_flags,
                          rel_flags ? rel_flags + r0 : nullptr, hs, A, true);
    c->grp_hwords = nullptr;
    c->grp_hstride = 0;
    c->grp_a0 = 0;
    if (rc) return rc;
    if (n_rel > 0 && rel_flags) HIPCHK(c, owgs_launch_relflags(rel_aid + r0, n_rel, out_invoker, rel_flags + r0, hs));
    // the context's health after the group: the last batch's (status bytes + bitmap, as owgs_update_health_device)
    if (status_dev) return update_health_device_impl(c, n_status, status_dev + (int64_t)(nb - 1) * status_stride, stream);
    return OWGS_OK;
}

int owgs_replay_device_group(owgs_ctx* c, int32_t n_batches, const int64_t* acq_off, const int64_t* rel_off,
                             const int32_t* act, const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker,
                             uint8_t* out_flags, uint8_t* rel_flags, const uint8_t* status_dev, int64_t status_stride,
                             int32_t n_status, void* stream) {
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    hipStream_t hs_ = stream ? (hipStream_t)stream : c->stream;
    int rc = order_on(c, hs_);
    if (!rc)
        rc = replay_device_group_impl(c, n_batches, acq_off, rel_off, act, rel_aid, seq_base, out_invoker, out_flags,
                                      rel_flags, status_dev, status_stride, n_status, stream);
    const int rt = tail_mark(c, hs_);
    return rc ? rc : rt;
}

static int replay_device_multi_impl(owgs_ctx** cs, int32_t k, const owgs_replay_io* io, void* stream) {
    if (!cs || !io || k < 1 || k > OWGS_MULTI_DEV_MAX) return OWGS_EINVAL;
    for (int32_t i = 0; i < k; ++i) {
        if (!cs[i]) return OWGS_EINVAL;
        if (cs[i]->cfg.device != cs[0]->cfg.device) return cs[0]->fail(OWGS_EINVAL, "shards on different devices");
        for (int32_t j = 0; j < i; ++j)
            if (cs[j] == cs[i]) return cs[0]->fail(OWGS_EINVAL, "one context twice in a multi-shard replay");
        if (io[i].n_batches <= 0) return cs[i]->fail(OWGS_EINVAL, "multi-shard replay needs batches in every shard");
    }
    hipStream_t hs = stream ? (hipStream_t)stream : cs[0]->stream;
    // every shard's engine in one launch needs one geometry and no watched pairs: the geometry each shard's launch
    // would take (lds_check applies the diagnostic override too)
    bool one_launch = true;
    for (int32_t i = 0; i < k; ++i) {
        // a shard on the large-state engine (its map and permits live in HBM, section 5.7) has no on-chip image to
        // launch with the others: every shard then replays through its own entry point, which routes it there
        if (cs[i]->large) {
            one_launch = false;
            continue;
        }
        const int rv = lds_check(cs[i]);
        if (rv) return rv;
        if (cs[i]->w_cap > 0 || cs[i]->variant != cs[0]->variant) one_launch = false;
    }
    if (!one_launch) {  // a shard in watch mode replays batch by batch (or geometries differ): every shard on its own
        for (int32_t j = 0; j < k; ++j) {
            const owgs_replay_io& x = io[j];
            int rc = replay_device_impl(cs[j], x.n_batches, x.acq_off, x.act, x.n_activations, x.rel_off, x.rel_aid,
                                        x.n_releases, x.seq_base, x.out_invoker, x.out_flags, x.rel_flags, hs);
            if (rc) return rc;
        }
        return OWGS_OK;
    }
    std::vector<OwgsEngineArgs> A((size_t)k);
    for (int32_t i = 0; i < k; ++i) {
        const owgs_replay_io& x = io[i];
        int rc = replay_begin(cs[i], x.n_batches, x.acq_off, x.act, x.n_activations, x.rel_off, x.rel_aid,
                              x.n_releases, x.seq_base, x.out_invoker, x.out_flags, x.rel_flags, hs, A[(size_t)i], false);
        if (rc) return rc;
    }
    for (int32_t i = 0; i < k; ++i) HIPCHK(cs[i], hipEventRecord(cs[i]->ev_engine[0], hs));
    if (k <= OWGS_MULTI_MAX) {
        HIPCHK(cs[0], cs[0]->variant ? owgs_launch_engine_multi_narrow(A.data(), k, hs)
                                     : owgs_launch_engine_multi(A.data(), k, hs));
    } else {  // argument blocks through HBM: the leader context's buffer, staged from its pinned host copy
        owgs_ctx* c0 = cs[0];
        const size_t bytes = (size_t)k * sizeof(OwgsEngineArgs);
        // the previous multi launch of this leader (maybe on another stream) may still read both buffers
        if (c0->ev_margs_valid) HIPCHK(c0, hipEventSynchronize(c0->ev_margs));
        if (c0->h_margs_bytes < bytes) {
            if (c0->h_margs) (void)hipHostFree(c0->h_margs);
            c0->h_margs = nullptr;
            c0->h_margs_bytes = 0;
            HIPCHK(c0, hipHostMalloc(&c0->h_margs, bytes, hipHostMallocDefault));
            c0->h_margs_bytes = bytes;
        }
        if (!c0->ev_margs) HIPCHK(c0, hipEventCreateWithFlags(&c0->ev_margs, hipEventDisableTiming));
        memcpy(c0->h_margs, A.data(), bytes);
        HIPCHK(c0, c0->d_margs.reserve((bytes + 3) / 4));
        HIPCHK(c0, hipMemcpyAsync(c0->d_margs.p, c0->h_margs, bytes, hipMemcpyHostToDevice, hs));
        HIPCHK(c0, c0->variant ? owgs_launch_engine_multi_dev_narrow(A.data(), (const OwgsEngineArgs*)c0->d_margs.p, k, hs)
                               : owgs_launch_engine_multi_dev(A.data(), (const OwgsEngineArgs*)c0->d_margs.p, k, hs));
        HIPCHK(c0, hipEventRecord(c0->ev_margs, hs));
        c0->ev_margs_valid = true;
    }
    for (int32_t i = 0; i < k; ++i) {
        HIPCHK(cs[i], hipEventRecord(cs[i]->ev_engine[1], hs));
        cs[i]->ev_engine_valid = true;
        const owgs_replay_io& x = io[i];
        if (x.rel_off && x.rel_flags)
            HIPCHK(cs[i], owgs_launch_relflags(x.rel_aid, x.n_releases, x.out_invoker, x.rel_flags, hs));
    }
    return OWGS_OK;
}

int owgs_replay_device_multi(owgs_ctx** cs, int32_t k, const owgs_replay_io* io, void* stream) {
    if (!cs || !io || k < 1 || k > OWGS_MULTI_DEV_MAX) return OWGS_EINVAL;
    for (int32_t i = 0; i < k; ++i)
        if (!cs[i]) return OWGS_EINVAL;
    (void)hipSetDevice(cs[0]->cfg.device);
    for (int32_t i = 0; i < k; ++i) {
        const int q = res_quiesce(cs[i]);
        if (q) return q;
    }
    hipStream_t hs_ = stream ? (hipStream_t)stream : cs[0]->stream;
    int rc = OWGS_OK;
    for (int32_t i = 0; i < k && !rc; ++i) rc = order_on(cs[i], hs_);
    if (!rc) rc = replay_device_multi_impl(cs, k, io, stream);
    for (int32_t i = 0; i < k; ++i) {
        const int rt = tail_mark(cs[i], hs_);
        if (!rc) rc = rt;
    }
    return rc;
}

static int replay_begin(owgs_ctx* c, int32_t n_batches, const int64_t* acq_off, const int32_t* act,
                        int64_t n_activations, const int64_t* rel_off, const int64_t* rel_aid, int64_t n_releases,
                        uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags, uint8_t* rel_flags,
                        hipStream_t hs, OwgsEngineArgs& A, bool launch) {
    if (!c || n_batches < 0 || !acq_off || !act || !out_invoker || !out_flags || n_activations < 0 ||
        n_activations >= ((int64_t)1 << 31) || n_releases < 0 || (n_releases > 0 && (!rel_off || !rel_aid)))
        return OWGS_EINVAL;
    if (n_batches == 0) return OWGS_OK;
    if (c->a_mem.empty()) return c->fail(OWGS_ENOENT, "no actions registered");
    OWGS_ENTER(c);
    base_args(c, A);
    A.seq_base = seq_base;
    A.out_inv = out_invoker;
    A.out_flags = out_flags;
    A.rel_flags = rel_flags;
    int rc = run_prepass(c, A, n_batches, acq_off, act, n_activations, hs);
    if (rc) return rc;
    if (rel_off) {
        // release bookkeeping: each released activation's release position; the engine writes the records
        const int64_t nr = std::max<int64_t>(n_releases, 1);
        HIPCHK(c, c->d_relx.reserve((size_t)std::max<int64_t>(n_activations, 1)));
        HIPCHK(c, c->d_rel_rec.reserve((size_t)nr));
        HIPCHK(c, hipMemsetAsync(c->d_relx.p, 0xFF, (size_t)n_activations * 4, hs));
        // a record no decision writes (device streams are not checked on the host: a release of a later activation)
        // reads as "no ActivationEntry"
        HIPCHK(c, hipMemsetAsync(c->d_rel_rec.p, 0xFF, (size_t)nr * sizeof(uint2), hs));
        if (rel_flags && n_releases) HIPCHK(c, hipMemsetAsync(rel_flags, 0, (size_t)n_releases, hs));
        HIPCHK(c, c->d_relcnt.reserve((size_t)2 * n_batches));
        HIPCHK(c, hipMemsetAsync(c->d_relcnt.p, 0, (size_t)2 * n_batches * 4, hs));
        OwgsRelposArgs ra{};
        ra.rel_aid = rel_aid;
        ra.n_rel = n_releases;
        ra.n_act = n_activations;
        ra.rel_off = rel_off;
        ra.n_batches = n_batches;
        ra.act = act;
        ra.act_meta = c->d_act_meta.p;
        ra.relx = c->d_relx.p;
        ra.relcnt = c->d_relcnt.p;
        ra.err = c->d_err.p;
        ra.decided_below = c->grp_a0;  // (group launches: earlier activations' records come from their decisions)
        ra.out_inv = out_invoker;
        ra.act_slot = c->d_act_slot.p;
        ra.rel_rec = c->d_rel_rec.p;
        HIPCHK(c, owgs_launch_relpos(&ra, hs));
        A.rel_off = rel_off;
        A.relpos = c->d_relx.p;
        A.relcnt = c->d_relcnt.p;
        A.rel_rec = c->d_rel_rec.p;
    }
    return run_engine(c, A, hs, launch);
}

int owgs_replay(owgs_ctx* c, int32_t n_batches, const int64_t* acq_off, const int32_t* act, const int64_t* rel_off,
                const int64_t* rel_aid, uint64_t seq_base, int32_t* out_invoker, uint8_t* out_flags,
                uint8_t* rel_flags) {
    if (!c || n_batches < 0 || !acq_off || !act || !out_invoker || !out_flags || !rel_off) return OWGS_EINVAL;
    if (n_batches == 0) return OWGS_OK;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    const int64_t n_act = acq_off[n_batches], n_rel = rel_off[n_batches];
    for (int32_t b = 0; b < n_batches; ++b)
        if (acq_off[b + 1] < acq_off[b] || rel_off[b + 1] < rel_off[b]) return c->fail(OWGS_EINVAL, "offsets");
    if (acq_off[0] != 0 || rel_off[0] != 0) return c->fail(OWGS_EINVAL, "offsets must start at 0");
    if (!registered(c, (int32_t)std::min<int64_t>(n_act, INT32_MAX), act)) return c->fail(OWGS_ENOENT, "unknown action");
    // a release refers to an activation of an earlier batch
    for (int32_t b = 0; b < n_batches; ++b)
        for (int64_t r = rel_off[b]; r < rel_off[b + 1]; ++r)
            if (rel_aid[r] < 0 || rel_aid[r] >= acq_off[b]) return c->fail(OWGS_EINVAL, "release id outside the stream");
    std::vector<int64_t> offs((size_t)2 * (n_batches + 1));
    memcpy(offs.data(), acq_off, (size_t)(n_batches + 1) * 8);
    memcpy(offs.data() + n_batches + 1, rel_off, (size_t)(n_batches + 1) * 8);
    HIPCHK(c, upload(c->d_off, offs.data(), offs.size(), c->stream));
    HIPCHK(c, upload(c->d_a, act, (size_t)n_act, c->stream));
    HIPCHK(c, upload(c->d_rel, rel_aid, (size_t)n_rel, c->stream));
    HIPCHK(c, c->d_out.reserve((size_t)n_act));
    HIPCHK(c, c->d_flags.reserve((size_t)n_act));
    HIPCHK(c, c->d_rflags.reserve((size_t)std::max<int64_t>(n_rel, 1)));
    int rc = owgs_replay_device(c, n_batches, c->d_off.p, c->d_a.p, n_act, c->d_off.p + n_batches + 1, c->d_rel.p,
                                n_rel, seq_base, c->d_out.p, c->d_flags.p, c->d_rflags.p, nullptr);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(out_invoker, c->d_out.p, (size_t)n_act * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out_flags, c->d_flags.p, (size_t)n_act, hipMemcpyDeviceToHost, c->stream));
    if (rel_flags && n_rel)
        HIPCHK(c, hipMemcpyAsync(rel_flags, c->d_rflags.p, (size_t)n_rel, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return check_err_word(c);
}

// One drained batch of the shim's batching thread: runs of completions then publishes.  One pinned
// H2D of every input, one launch chain (release staging, pre-pass, ONE engine launch over all runs), one pinned D2H
// of every output, one synchronisation.  With watched pairs (owgs_watch.hip) the runs go through the exact release
// kernels, one engine launch per run and the watch update instead -- still one copy each way and one sync.
// The per-run path of owgs_process_batch (watched pairs, a call of completions only, or a fused call whose releases
// could leave the engine's permit range): per run the exact release kernels (ForcibleSemaphore's overflow Error per
// release, FS:48-50), then an engine launch for its publishes and, with watched pairs, the watch update.
static int process_runs(owgs_ctx* c, int32_t n_runs, const int32_t* rel_off, const int32_t* pub_off, const int64_t* d_run,
                        const int32_t* d_pa, const int32_t* d_ri, const int32_t* d_ra, const u64* d_sq,
                        uint64_t seq_base, int32_t* d_out, uint8_t* d_fl, uint8_t* d_rf, hipStream_t s) {
    int rc = OWGS_OK;
    int32_t max_r = 1;
    for (int32_t r = 0; r < n_runs; ++r) max_r = std::max(max_r, rel_off[r + 1] - rel_off[r]);
    HIPCHK(c, c->w_rel.reserve((size_t)3 * max_r));
    int32_t* q = c->w_rel.p;
    for (int32_t r = 0; r < n_runs && !rc; ++r) {
        const int32_t nr = rel_off[r + 1] - rel_off[r], np = pub_off[r + 1] - pub_off[r];
        if (nr > 0) {
            HIPCHK(c, owgs_launch_relmeta(nr, d_ra + rel_off[r], c->d_act_mem.p, c->d_act_maxc.p, c->d_act_slot.p, q,
                                          q + max_r, q + 2 * max_r, s));
            rc = release_chain(c, nr, d_ri + rel_off[r], q, q + max_r, q + 2 * max_r, d_rf + rel_off[r], s);
        }
        if (!rc && np > 0) {
            OwgsEngineArgs A;
            base_args(c, A);
            A.seq_base = seq_base + (uint64_t)pub_off[r];
            A.seq = d_sq ? d_sq + pub_off[r] : nullptr;
            A.out_inv = d_out + pub_off[r];
            A.out_flags = d_fl + pub_off[r];
            rc = run_prepass(c, A, 1, d_run + 2 * r, d_pa + pub_off[r], np, s);
            if (!rc) rc = run_engine(c, A, s);
            if (!rc) rc = w_update(c, np, d_pa + pub_off[r], d_out + pub_off[r], d_fl + pub_off[r], s);
        }
    }
    return rc;
}

// One drained batch of the shim's batching thread: runs of completions then publishes.  One pinned
// H2D of every input, one launch chain (release staging, pre-pass, ONE engine launch over all runs), one pinned D2H
// of every output, one synchronisation.  With watched pairs (owgs_watch.hip) the runs go through the exact release
// kernels, one engine launch per run and the watch update instead -- still one copy each way and one sync.
int owgs_process_batch(owgs_ctx* c, int32_t n_runs, const int32_t* rel_off, const int32_t* rel_invoker,
                       const int32_t* rel_action, uint8_t* rel_flags, const int32_t* pub_off,
                       const int32_t* pub_action, const uint64_t* seq, uint64_t seq_base, int32_t* out_invoker,
                       uint8_t* out_flags) {
    const CallTimer timer_(c);
    if (!c || n_runs < 0 || (n_runs > 0 && (!rel_off || !pub_off))) return OWGS_EINVAL;
    if (n_runs == 0) return OWGS_OK;
    if (rel_off[0] != 0 || pub_off[0] != 0) return c->fail(OWGS_EINVAL, "offsets must start at 0");
    for (int32_t r = 0; r < n_runs; ++r)
        if (rel_off[r + 1] < rel_off[r] || pub_off[r + 1] < pub_off[r]) return c->fail(OWGS_EINVAL, "offsets");
    const int32_t NR = rel_off[n_runs], NP = pub_off[n_runs];
    if ((NR > 0 && (!rel_invoker || !rel_action)) || (NP > 0 && (!pub_action || !out_invoker || !out_flags)))
        return OWGS_EINVAL;
    if (n_runs >= 0x1FFFF) return c->fail(OWGS_ERANGE, "more than 131070 runs in one call");
    if (!registered(c, NP, pub_action) || !registered(c, NR, rel_action)) return c->fail(OWGS_ENOENT, "unknown action");
    (void)hipSetDevice(c->cfg.device);  // (the resident engine is stopped below only when the chain takes the call)
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    hipStream_t s = c->stream;
    // explicit sequence numbers that count up from the first one are the implicit form (seq_base + i): the engine's
    // specialisations without the per-activation sequence loads then take the call (the shim numbers its publishes
    // in queue order)
    if (seq && NP > 0) {
        bool consecutive = true;
        for (int32_t i = 1; i < NP && consecutive; ++i) consecutive = seq[i] == seq[0] + (uint64_t)i;
        if (consecutive) {
            seq_base = seq[0];
            seq = nullptr;
        }
    }
    if (c->large)
        return seq_host_runs(c, n_runs, rel_off, rel_invoker, rel_action, rel_flags, pub_off, pub_action, seq,
                             seq_base, out_invoker, out_flags);
    // small calls: the resident engine (owgs_resident.hip), no launch, copy or synchronisation per call
    if (res_eligible(c, n_runs, NR, NP, seq != nullptr)) {
        int served = 0;
        const int rr = res_process(c, n_runs, rel_off, rel_invoker, rel_action, rel_flags, pub_off, pub_action, seq,
                                   seq_base, out_invoker, out_flags, &served);
        if (rr || served) {
            c->res_last_served = served != 0;
            return rr;
        }
    }
    const bool relaunch = c->res_last_served && env_opts().res_eager > 0;
    c->res_last_served = false;
    {
        const int q = res_quiesce(c);
        if (q) return q;
    }
    ++c->res_n_chained;
    // ---- pinned staging: i64 offsets (publishes, releases, per-run {0, n}) | publish actions | release invokers |
    // release actions | seq
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t o_acq = 0, o_rel = al(o_acq + 8 * (size_t)(n_runs + 1)), o_run = al(o_rel + 8 * (size_t)(n_runs + 1));
    const size_t o_pa = al(o_run + 16 * (size_t)n_runs), o_ri = al(o_pa + 4 * (size_t)NP);
    const size_t o_ra = al(o_ri + 4 * (size_t)NR), o_sq = al(o_ra + 4 * (size_t)NR);
    const size_t in_bytes = al(o_sq + (seq ? 8 * (size_t)NP : 0));
    const size_t q_inv = 0, q_fl = al(4 * (size_t)NP), q_rf = al(q_fl + (size_t)NP), q_err = al(q_rf + (size_t)NR);
    const size_t out_bytes = q_err + 16;
    if (c->h_pin_bytes < in_bytes) {
        if (c->h_pin) (void)hipHostFree(c->h_pin);
        c->h_pin = nullptr;
        c->h_pin_bytes = 0;
        HIPCHK(c, hipHostMalloc(&c->h_pin, in_bytes * 2, hipHostMallocDefault));
        c->h_pin_bytes = in_bytes * 2;
    }
    if (c->h_pout_bytes < out_bytes) {
        if (c->h_pout) (void)hipHostFree(c->h_pout);
        c->h_pout = nullptr;
        c->h_pout_bytes = 0;
        HIPCHK(c, hipHostMalloc(&c->h_pout, out_bytes * 2, hipHostMallocDefault));
        c->h_pout_bytes = out_bytes * 2;
    }
    HIPCHK(c, hipStreamSynchronize(s));  // the previous call's copies out of the pinned buffers are done
    char* H = (char*)c->h_pin;
    int64_t* h_acq = (int64_t*)(H + o_acq);
    int64_t* h_rel = (int64_t*)(H + o_rel);
    int64_t* h_run = (int64_t*)(H + o_run);
    for (int32_t r = 0; r <= n_runs; ++r) {
        h_acq[r] = pub_off[r];
        h_rel[r] = rel_off[r];
    }
    for (int32_t r = 0; r < n_runs; ++r) {
        h_run[2 * r] = 0;
        h_run[2 * r + 1] = pub_off[r + 1] - pub_off[r];
    }
    if (NP) memcpy(H + o_pa, pub_action, 4 * (size_t)NP);
    if (NR) {
        memcpy(H + o_ri, rel_invoker, 4 * (size_t)NR);
        memcpy(H + o_ra, rel_action, 4 * (size_t)NR);
    }
    if (seq && NP) memcpy(H + o_sq, seq, 8 * (size_t)NP);
    bool fused = !(c->w_cap > 0 || NP == 0);
    // a fused call's kernels (release staging, pre-pass, engine) read the inputs from the pinned block itself, over
    // PCIe: no host-to-device copy, and no wait for it before the first kernel.  The per-run path copies them to HBM.
    char* D = H;
    auto to_hbm = [&]() -> int {
        HIPCHK(c, c->d_pin.reserve(in_bytes));
        HIPCHK(c, hipMemcpyAsync(c->d_pin.p, H, in_bytes, hipMemcpyHostToDevice, s));
        D = (char*)c->d_pin.p;
        return OWGS_OK;
    };
    if (!fused) {
        const int rh = to_hbm();
        if (rh) return rh;
    }
    const int64_t* d_acq = (const int64_t*)(D + o_acq);
    const int64_t* d_rel = (const int64_t*)(D + o_rel);
    const int64_t* d_run = (const int64_t*)(D + o_run);
    const int32_t* d_pa = (const int32_t*)(D + o_pa);
    const int32_t* d_ri = (const int32_t*)(D + o_ri);
    const int32_t* d_ra = (const int32_t*)(D + o_ra);
    const u64* d_sq = seq ? (const u64*)(D + o_sq) : nullptr;
    HIPCHK(c, c->d_pout.reserve(out_bytes));
    char* DO = (char*)c->d_pout.p;
    int32_t* d_out = (int32_t*)(DO + q_inv);
    uint8_t* d_fl = (uint8_t*)(DO + q_fl);
    uint8_t* d_rf = (uint8_t*)(DO + q_rf);
    int rc = OWGS_OK;
    if (!fused) {
        // watched pairs: the exact release kernels per run, the watch update after each publish run; a call of
        // completions only: the release kernels alone (cheaper than an engine launch)
        rc = process_runs(c, n_runs, rel_off, pub_off, d_run, d_pa, d_ri, d_ra, d_sq, seq_base, d_out, d_fl, d_rf, s);
    } else {  // every run in ONE engine launch: the releases as engine records (owgs_fused.hip)
        if (c->a_mem.empty()) return c->fail(OWGS_ENOENT, "no actions registered");
        HIPCHK(c, c->f_rec.reserve((size_t)NR + 2));
        HIPCHK(c, c->f_src.reserve((size_t)NR + 1));
        HIPCHK(c, c->f_cnt.reserve((size_t)2 * n_runs));
        if (c->f_bound.n < (size_t)std::max(c->n_slots, 1)) {  // zero between calls (the engine clears what it reads)
            HIPCHK(c, c->f_bound.reserve((size_t)std::max(c->n_slots, 1)));
            HIPCHK(c, hipMemsetAsync(c->f_bound.p, 0, c->f_bound.n * 8, s));
        }
        if (NR > 0) {
            OwgsStageArgs g{};
            g.n_runs = n_runs;
            g.rel_off = d_rel;
            g.rel_inv = d_ri;
            g.rel_act = d_ra;
            g.act_mem = c->d_act_mem.p;
            g.act_maxc = c->d_act_maxc.p;
            g.act_slot = c->d_act_slot.p;
            g.n_slots = c->n_slots;
            g.rel_rec = c->f_rec.p;
            g.rel_src = c->f_src.p;
            g.relcnt = c->f_cnt.p;
            g.rel_flags = d_rf;
            g.bound = c->f_bound.p;
            HIPCHK(c, owgs_launch_stage_releases(&g, s));
        }
        OwgsEngineArgs A;
        base_args(c, A);
        A.seq_base = seq_base;
        A.seq = d_sq;
        A.out_inv = d_out;
        A.out_flags = d_fl;
        rc = run_prepass(c, A, n_runs, d_acq, d_pa, NP, s);
        if (!rc && NR > 0) {
            A.rel_off = d_rel;
            A.relcnt = c->f_cnt.p;
            A.rel_rec = c->f_rec.p;
            A.rel_src = c->f_src.p;
            A.rel_flags = d_rf;
            A.rel_bound = c->f_bound.p;
        }
        // the context's error word after the launch: stored by the engine into the pinned output block (past the
        // range the copy below brings back), not copied after it
        A.err_host = (int32_t*)((char*)c->h_pout + q_err);
        // ... and its outputs: the engine's last step copies them there (no copy queued behind it)
        A.out_copy_src = (const uint4*)c->d_pout.p;
        A.out_copy_dst = (uint4*)c->h_pout;
        A.out_copy_n16 = (int32_t)(q_err / 16);
        if (!rc) rc = run_engine(c, A, s);
    }
    if (rc) return rc;
    if (!fused) {
        HIPCHK(c, hipMemcpyAsync(c->d_pout.p + q_err, c->d_err.p, 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->h_pout, c->d_pout.p, out_bytes, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(c, hipStreamSynchronize(s));
    const char* HO = (const char*)c->h_pout;
    int32_t e = 0;
    memcpy(&e, HO + q_err, 4);
    if (fused && (e & OWGS_ERR_RELRISK)) {
        // the releases could push a slot out of the engine's range: the engine stopped before touching anything, so
        // the call runs again through the per-run path, whose release kernels apply ForcibleSemaphore's bound
        // release by release (FS:48-50) exactly as owgs_release_batch does
        HIPCHK(c, hipMemsetAsync(c->d_err.p, 0, sizeof(int32_t), s));
        HIPCHK(c, hipMemsetAsync(c->f_bound.p, 0, c->f_bound.n * 8, s));
        if (D == H) {  // (the per-run path reads its inputs from HBM)
            const int rh = to_hbm();
            if (rh) return rh;
            d_acq = (const int64_t*)(D + o_acq);
            d_rel = (const int64_t*)(D + o_rel);
            d_run = (const int64_t*)(D + o_run);
            d_pa = (const int32_t*)(D + o_pa);
            d_ri = (const int32_t*)(D + o_ri);
            d_ra = (const int32_t*)(D + o_ra);
            d_sq = seq ? (const u64*)(D + o_sq) : nullptr;
        }
        rc = process_runs(c, n_runs, rel_off, pub_off, d_run, d_pa, d_ri, d_ra, d_sq, seq_base, d_out, d_fl, d_rf, s);
        if (rc) return rc;
        HIPCHK(c, hipMemcpyAsync(c->d_pout.p + q_err, c->d_err.p, 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->h_pout, c->d_pout.p, out_bytes, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        memcpy(&e, HO + q_err, 4);
    }
    if (NP) {
        memcpy(out_invoker, HO + q_inv, 4 * (size_t)NP);
        memcpy(out_flags, HO + q_fl, (size_t)NP);
    }
    if (NR && rel_flags) memcpy(rel_flags, HO + q_rf, (size_t)NR);
    rc = w_refresh(c, s);
    if (rc) return rc;
    if (e) return check_err_word(c);
    // small calls came before this one: launch the resident engine again now, so that it loads the state while the
    // host returns instead of the next small call paying the launch and the load.  Only here, after this call's
    // stream has drained: an operation queued behind the engine on a hardware queue the streams share would wait for
    // its idle exit
    if (relaunch && res_eligible(c, 1, 0, 1, false) && c->res_in && c->res_out && !c->res_alive) {
        const int rl = res_launch(c);
        if (rl) return rl;
    }
    return OWGS_OK;
}

int owgs_snapshot(owgs_ctx* c) {
    if (!c) return OWGS_EINVAL;
    OWGS_NOT_LARGE(c);
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    HIPCHK(c, c->s_permits.reserve((size_t)std::max(c->n_slots, 1)));
    HIPCHK(c, c->s_ct_keys.reserve(OWGS_CTC));
    HIPCHK(c, c->s_ct_vals.reserve(OWGS_CTC));
    if (c->n_slots)
        HIPCHK(c, hipMemcpyAsync(c->s_permits.p, c->d_permits.p, (size_t)c->n_slots * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->s_ct_keys.p, c->d_ct_keys.p, OWGS_CTC * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->s_ct_vals.p, c->d_ct_vals.p, OWGS_CTC * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->s_ovf_cnt = 0;
    if (c->ovf_cap > 0) {  // the overflow part of the map, when it holds entries
        HIPCHK(c, hipMemcpy(&c->s_ovf_cnt, c->d_ovf_cnt.p, sizeof(int32_t), hipMemcpyDeviceToHost));
        if (c->s_ovf_cnt > 0) {
            HIPCHK(c, c->s_ovf.reserve((size_t)c->ovf_cap));
            HIPCHK(c, hipMemcpy(c->s_ovf.p, c->d_ovf.p, (size_t)c->ovf_cap * sizeof(uint2), hipMemcpyDeviceToDevice));
            c->s_ovf_cap = c->ovf_cap;
        }
    }
    c->s_w_cap = c->w_cap;  // watched pairs
    c->s_w_live = c->w_live;
    if (c->w_cap > 0) {
        HIPCHK(c, c->s_w_keys.reserve((size_t)c->w_cap));
        HIPCHK(c, c->s_w_vals.reserve((size_t)c->w_cap));
        HIPCHK(c, c->s_w_wkey.reserve((size_t)OWGS_MAX_SLOTKEYS + 1));
        HIPCHK(c, hipMemcpy(c->s_w_keys.p, c->w_keys.p, (size_t)c->w_cap * 4, hipMemcpyDeviceToDevice));
        HIPCHK(c, hipMemcpy(c->s_w_vals.p, c->w_vals.p, (size_t)c->w_cap * 4, hipMemcpyDeviceToDevice));
        HIPCHK(c, hipMemcpy(c->s_w_wkey.p, c->w_wkey.p, ((size_t)OWGS_MAX_SLOTKEYS + 1) * 4, hipMemcpyDeviceToDevice));
    }
    c->has_snap = true;
    c->snap_slots = c->n_slots;
    c->snap_slot_epoch = c->slot_epoch;
    return OWGS_OK;
}

static int restore_impl(owgs_ctx* c, void* stream) {
    if (!c || !c->has_snap || c->snap_slots != c->n_slots) return OWGS_EINVAL;
    OWGS_NOT_LARGE(c);
    // a key recycled since the snapshot may name another fqn@version now: the snapshot's entries would alias it
    if (c->slot_epoch != c->snap_slot_epoch) return c->fail(OWGS_EINVAL, "keys were recycled since the snapshot");
    OWGS_ENTER(c);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (c->n_slots)
        HIPCHK(c, hipMemcpyAsync(c->d_permits.p, c->s_permits.p, (size_t)c->n_slots * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_ct_keys.p, c->s_ct_keys.p, OWGS_CTC * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_ct_vals.p, c->s_ct_vals.p, OWGS_CTC * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, hipMemsetAsync(c->d_clast.p, 0, sizeof(int32_t), s));  // (the replays after a restore start alike)
    if (c->ovf_cap > 0) {
        const OwgsOvf O = ovf_args(c);
        if (c->s_ovf_cnt > 0 && c->s_ovf_cap == c->ovf_cap) {
            HIPCHK(c, hipMemcpyAsync(c->d_ovf.p, c->s_ovf.p, (size_t)c->ovf_cap * sizeof(uint2), hipMemcpyDeviceToDevice, s));
            HIPCHK(c, hipMemcpyAsync(c->d_ovf_cnt.p, &c->s_ovf_cnt, sizeof(int32_t), hipMemcpyHostToDevice, s));
        } else {
            HIPCHK(c, owgs_launch_ovf_clear(&O, s));  // (a no-op kernel while the overflow is empty)
            if (c->s_ovf_cnt > 0)  // the table grew since the snapshot: its entries are rehashed
                HIPCHK(c, owgs_launch_ovf_rehash(c->s_ovf.p, c->s_ovf_cap, &O, c->d_err.p, s));
        }
    }
    c->ovf_used_ub = c->s_ovf_cnt;
    ovf_probes_clear(c);
    if (c->w_cap != c->s_w_cap) {  // watched pairs as captured
        w_drop(c);
        if (c->s_w_cap > 0) {
            HIPCHK(c, c->w_keys.reserve((size_t)c->s_w_cap));
            HIPCHK(c, c->w_vals.reserve((size_t)c->s_w_cap));
            HIPCHK(c, c->w_wkey.reserve((size_t)OWGS_MAX_SLOTKEYS + 1));
            HIPCHK(c, c->w_cnt.reserve(1));
        }
    }
    if (c->s_w_cap > 0) {
        HIPCHK(c, hipMemcpyAsync(c->w_keys.p, c->s_w_keys.p, (size_t)c->s_w_cap * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->w_vals.p, c->s_w_vals.p, (size_t)c->s_w_cap * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->w_wkey.p, c->s_w_wkey.p, ((size_t)OWGS_MAX_SLOTKEYS + 1) * 4,
                                 hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->w_cnt.p, &c->s_w_live, sizeof(int32_t), hipMemcpyHostToDevice, s));
        c->w_cap = c->s_w_cap;
        c->w_live = c->s_w_live;
    }
    return OWGS_OK;
}

int owgs_restore(owgs_ctx* c, void* stream) {
    if (c) ++c->res_cache_epoch;
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    hipStream_t hs_ = stream ? (hipStream_t)stream : c->stream;
    int rc = order_on(c, hs_);
    if (!rc) rc = restore_impl(c, stream);
    const int rt = tail_mark(c, hs_);  // (also after a failure: whatever was enqueued stays ordered)
    return rc ? rc : rt;
}

static int update_health_device_impl(owgs_ctx* c, int32_t n, const uint8_t* status_dev, void* stream) {
    if (!c || n != (int32_t)c->status.size() || (n > 0 && !status_dev)) return OWGS_EINVAL;
    OWGS_ENTER(c);
    if (n && c->pool_mode == 0 && !c->pool_override[0] && !c->pool_override[1] && c->d_status.p && c->d_usable.p) {
        // identity pools (position = id): health changes only the usable bitmap, and the engine counts the healthy
        // invokers of each pool from it (the overload fallback's |H|, SCPB:417-424).  Nothing else depends on the
        // status, so the update stays on the stream: the status bytes, the bitmap, and the host mirror later.
        hipStream_t s = stream ? (hipStream_t)stream : c->stream;
        HIPCHK(c, hipMemcpyAsync(c->d_status.p, status_dev, (size_t)n, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, owgs_launch_usable(c->d_status.p, n, c->d_usable.p, (n + 31) / 32 + 1, s));
        if (!c->ev_status) HIPCHK(c, hipEventCreateWithFlags(&c->ev_status, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(c->ev_status, s));
        c->status_stale = true;
        return OWGS_OK;
    }
    int rs = sync_status(c);
    if (rs) return rs;
    if (n) {
        HIPCHK(c, hipMemcpyAsync(c->status.data(), status_dev, (size_t)n, hipMemcpyDeviceToHost,
                                 stream ? (hipStream_t)stream : c->stream));
        HIPCHK(c, hipMemcpyAsync(c->d_status.p, status_dev, (size_t)n, hipMemcpyDeviceToDevice,
                                 stream ? (hipStream_t)stream : c->stream));
        HIPCHK(c, hipStreamSynchronize(stream ? (hipStream_t)stream : c->stream));
    }
    int rc = rebuild_pools(c);
    if (!rc) HIPCHK(c, hipStreamSynchronize(c->stream));
    return rc;
}

int owgs_update_health_device(owgs_ctx* c, int32_t n, const uint8_t* status_dev, void* stream) {
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    hipStream_t hs_ = stream ? (hipStream_t)stream : c->stream;
    int rc = order_on(c, hs_);
    if (!rc) rc = update_health_device_impl(c, n, status_dev, stream);
    const int rt = tail_mark(c, hs_);  // (also after a failure: whatever was enqueued stays ordered)
    return rc ? rc : rt;
}

int owgs_selftest(owgs_ctx* c) {
    if (!c) return OWGS_EINVAL;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    HIPCHK(c, hipMemsetAsync(c->d_err.p, 0, sizeof(int32_t), c->stream));
    HIPCHK(c, owgs_launch_selftest(c->d_err.p, 64, c->stream));
    int32_t bad = 0;
    HIPCHK(c, hipMemcpyAsync(&bad, c->d_err.p, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_err.p, 0, sizeof(int32_t), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return bad ? c->fail(OWGS_EDEVICE, "device self-test mismatch") : OWGS_OK;
}

int owgs_read_stats(owgs_ctx* c, uint64_t* out, int32_t cap) {
    if (!c || !out) return OWGS_EINVAL;
    // a live resident engine is stopped first (it writes the state back): a copy on the context's stream could
    // otherwise sit behind it on a hardware queue the two streams share until its idle exit
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    u64 v[OWGS_NSTATS];
    HIPCHK(c, hipMemcpyAsync(v, c->d_stats.p + (size_t)c->stats_last * OWGS_NSTATS, sizeof(v), hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->large) {  // (the large-state engine keeps no device counters: its decisions by path, since the context began)
        v[46] = (u64)c->q_spec;
        v[47] = (u64)c->q_alone;
        for (int k = 0; k < 4; ++k) v[40 + k] = c->q_cyc[k];
    }
    for (int32_t i = 0; i < cap && i < OWGS_NSTATS; ++i) out[i] = v[i];
    return OWGS_OK;
}

}  // extern "C"

// ============================================================================================== completion acks
// activationSlots (CLB:60) on the device; see owgs_acks.hip.

static OwgsActTable act_table(owgs_ctx* c) {
    OwgsActTable T;
    T.tw = c->t_tw.p;
    T.tk = c->t_tk.p;
    T.tv = c->t_tv.p;
    T.owner = c->t_owner.p;
    T.cap = c->t_cap;
    return T;
}

// keep used slots (live + deleted) under half the capacity: rehash the live entries into a table of
// max(cap, 4 * (live + n)) slots when n more inserts could cross it
static int act_reserve(owgs_ctx* c, long long n) {
    if (c->t_cap > 0 && c->t_used + n <= c->t_cap / 2) return OWGS_OK;
    long long cap = 1 << 16;
    while (cap < 4 * (c->t_live + n)) cap <<= 1;
    if (cap < c->t_cap) cap = c->t_cap;
    DevBuf<unsigned long long> tw;
    DevBuf<ulonglong2> tk;
    DevBuf<int2> tv;
    DevBuf<int32_t> ow;
    HIPCHK(c, tw.reserve((size_t)cap));
    HIPCHK(c, tk.reserve((size_t)cap));
    HIPCHK(c, tv.reserve((size_t)cap));
    HIPCHK(c, ow.reserve((size_t)cap));
    OwgsActTable T{tw.p, tk.p, tv.p, ow.p, cap};
    HIPCHK(c, owgs_launch_act_init(&T, c->stream));
    if (c->t_cap > 0) {
        OwgsActTable O = act_table(c);
        HIPCHK(c, owgs_launch_act_rehash(&O, &T, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->t_tw.release();
    c->t_tk.release();
    c->t_tv.release();
    c->t_owner.release();
    c->t_tw = tw;
    c->t_tk = tk;
    c->t_tv = tv;
    c->t_owner = ow;
    tw.p = nullptr;
    tk.p = nullptr;
    tv.p = nullptr;
    ow.p = nullptr;
    c->t_cap = cap;
    c->t_used = c->t_live;
    return OWGS_OK;
}

int owgs_set_health_tid(owgs_ctx* c, int64_t start_ms) {
    if (!c) return OWGS_EINVAL;
    c->health_ms = start_ms;
    return OWGS_OK;
}

int owgs_activations_live(owgs_ctx* c, int64_t* live) {
    if (!c || !live) return OWGS_EINVAL;
    *live = c->t_live;
    return OWGS_OK;
}

int owgs_track_activations(owgs_ctx* c, int32_t n, const char* aid32, const int32_t* action, const int32_t* ticket,
                           int32_t* out_ticket, uint8_t* out_existed) {
    if (!c || n < 0 || (n > 0 && (!aid32 || !action || !ticket || !out_ticket || !out_existed))) return OWGS_EINVAL;
    if (n == 0) return OWGS_OK;
    if (!registered(c, n, action)) return c->fail(OWGS_ENOENT, "unknown action");
    // ActivationId.asString is 32 chars of [0-9a-f]; reject a malformed batch before any entry is created
    for (size_t k = 0; k < (size_t)n * 32; ++k) {
        const char ch = aid32[k];
        if (!((ch >= '0' && ch <= '9') || (ch >= 'a' && ch <= 'f')))
            return c->fail(OWGS_EINVAL, "activation id is not 32 characters of [0-9a-f]");
    }
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    int rc = act_reserve(c, n);
    if (rc) return rc;
    HIPCHK(c, upload(c->k_aid, aid32, (size_t)n * 32, c->stream));
    HIPCHK(c, upload(c->k_act, action, (size_t)n, c->stream));
    HIPCHK(c, upload(c->k_r0, ticket, (size_t)n, c->stream));
    HIPCHK(c, c->k_key.reserve((size_t)n));
    HIPCHK(c, c->k_slot.reserve((size_t)n));
    HIPCHK(c, c->k_state.reserve((size_t)n));
    HIPCHK(c, c->k_tick.reserve((size_t)n));
    HIPCHK(c, c->k_oflags.reserve((size_t)n));
    HIPCHK(c, c->k_cnt.reserve(2));
    HIPCHK(c, hipMemsetAsync(c->k_cnt.p, 0, 16, c->stream));
    HIPCHK(c, owgs_launch_aid_decode(c->k_aid.p, n, nullptr, c->k_key.p, nullptr, nullptr, nullptr, c->stream));
    OwgsActTable T = act_table(c);
    HIPCHK(c, owgs_launch_act_track(&T, c->k_key.p, n, c->k_act.p, c->k_r0.p, c->k_slot.p, c->k_state.p, c->k_tick.p,
                                    c->k_oflags.p, c->k_cnt.p, c->stream));
    unsigned long long cnt[2];
    HIPCHK(c, hipMemcpyAsync(out_ticket, c->k_tick.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out_existed, c->k_oflags.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(cnt, c->k_cnt.p, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->t_used += (long long)cnt[0];
    c->t_live += (long long)cnt[0];
    for (int32_t i = 0; i < n; ++i)
        if (out_existed[i] == 2) return c->fail(OWGS_EINVAL, "activation id is not 32 characters of [0-9a-f]");
    return OWGS_OK;
}

// shared tail: info/key/inst of n messages are in k_info/k_key/k_inst; resolve, release in order, flags
static int ack_complete(owgs_ctx* c, int32_t n, uint8_t* d_kind, int32_t* d_ticket, uint8_t* d_flags,
                        hipStream_t st) {
    if (c->t_cap == 0) {
        int rc = act_reserve(c, 0);
        if (rc) return rc;
    }
    HIPCHK(c, c->k_slot.reserve((size_t)n));
    HIPCHK(c, c->k_r0.reserve((size_t)n));
    HIPCHK(c, c->k_r1.reserve((size_t)n));
    HIPCHK(c, c->k_r2.reserve((size_t)n));
    HIPCHK(c, c->k_r3.reserve((size_t)n));
    HIPCHK(c, c->d_rflags.reserve((size_t)n));
    HIPCHK(c, c->k_cnt.reserve(2));
    HIPCHK(c, hipMemsetAsync(c->k_cnt.p, 0, 16, st));
    if (!c->d_act_mem.p) {  // no actions registered: every lookup misses, the records are never read
        HIPCHK(c, c->d_act_mem.reserve(1));
        HIPCHK(c, c->d_act_maxc.reserve(1));
        HIPCHK(c, c->d_act_slot.reserve(1));
    }
    OwgsActTable T = act_table(c);
    OwgsAckCompleteArgs a{};
    a.key = c->k_key.p;
    a.info = c->k_info.p;
    a.inst = c->k_inst.p;
    a.n = n;
    a.slot = c->k_slot.p;
    a.act_mem = c->d_act_mem.p;
    a.act_maxc = c->d_act_maxc.p;
    a.act_slot = c->d_act_slot.p;
    a.n_slots = c->n_slots;
    a.r_inv = c->k_r0.p;
    a.r_mem = c->k_r1.p;
    a.r_maxc = c->k_r2.p;
    a.r_slot = c->k_r3.p;
    a.out_kind = d_kind;
    a.out_ticket = d_ticket;
    a.counters = c->k_cnt.p;
    HIPCHK(c, owgs_launch_ack_complete(&T, &a, st));
    if (c->large) {  // the large-state engine applies the records in message order (owgs_seq.hip)
        const int64_t offs[4] = {0, (int64_t)n, 0, 0};
        HIPCHK(c, upload(c->g_off, offs, 4, st));
        OwgsSeqArgs S = seq_args(c);
        S.n_runs = 1;
        S.rel_off = c->g_off.p;
        S.pub_off = c->g_off.p + 2;
        S.rel_inv = c->k_r0.p;
        S.rel_mem = c->k_r1.p;
        S.rel_maxc = c->k_r2.p;
        S.rel_slot = c->k_r3.p;
        S.rel_flags = c->d_rflags.p;
        int rs = seq_run(c, S, st);
        if (rs) return rs;
        HIPCHK(c, owgs_launch_ack_flags(n, c->k_info.p, c->d_rflags.p, d_kind, d_flags, st));
        unsigned long long cnt[2];
        HIPCHK(c, hipMemcpyAsync(cnt, c->k_cnt.p, 16, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        c->t_live -= (long long)cnt[1];
        return check_err_word(c);
    }
    OwgsReleaseArgs R{};
    R.permits = c->d_permits.p;
    R.n_slots = c->n_slots;
    R.ct_keys = c->d_ct_keys.p;
    R.ct_vals = c->d_ct_vals.p;
    R.ovf = ovf_args(c);
    R.n = n;
    R.inv = c->k_r0.p;
    R.mem = c->k_r1.p;
    R.maxc = c->k_r2.p;
    R.slot = c->k_r3.p;
    R.flags = c->d_rflags.p;
    R.err = c->d_err.p;
    int rs = release_scratch(c, R, n);
    if (!rs && c->w_cap > 0) {
        rs = ensure_ovf(c, n, st);
        ovf_add(c, n);
    }
    if (rs) return rs;
    R.ovf = ovf_args(c);
    R.w = watch_args(c);
    HIPCHK(c, owgs_launch_release_seq(&R, st));
    HIPCHK(c, owgs_launch_ack_flags(n, c->k_info.p, c->d_rflags.p, d_kind, d_flags, st));
    unsigned long long cnt[2];
    HIPCHK(c, hipMemcpyAsync(cnt, c->k_cnt.p, 16, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    c->t_live -= (long long)cnt[1];
    rs = w_refresh(c, st);
    return rs ? rs : check_err_word(c);
}

int owgs_process_acks_device(owgs_ctx* c, int32_t n, const uint8_t* bytes, const int64_t* off, uint8_t* out_kind,
                             int32_t* out_invoker, int32_t* out_ticket, uint8_t* out_flags, void* stream) {
    if (!c || n < 0 || (n > 0 && (!bytes || !off || !out_kind || !out_invoker || !out_ticket || !out_flags)))
        return OWGS_EINVAL;
    if (n == 0) return OWGS_OK;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, stream ? (hipStream_t)stream : c->stream);
        if (ro_) return ro_;
    }
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(c, c->k_key.reserve((size_t)n));
    HIPCHK(c, c->k_info.reserve((size_t)n));
    OwgsAckParseArgs p{};
    p.bytes = bytes;
    p.off = off;
    p.n = n;
    p.health_start_ms = c->health_ms;
    p.forced = nullptr;
    p.key = c->k_key.p;
    p.inst = out_invoker;
    p.info = c->k_info.p;
    HIPCHK(c, owgs_launch_ack_parse(&p, st));
    // the resolve step reads the instance from k_inst
    HIPCHK(c, c->k_inst.reserve((size_t)n));
    HIPCHK(c, hipMemcpyAsync(c->k_inst.p, out_invoker, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
    return ack_complete(c, n, out_kind, out_ticket, out_flags, st);
}

int owgs_process_acks(owgs_ctx* c, int32_t n, const char* bytes, const int64_t* off, uint8_t* out_kind,
                      int32_t* out_invoker, int32_t* out_ticket, uint8_t* out_flags) {
    if (!c || n < 0 || (n > 0 && (!bytes || !off || !out_kind || !out_invoker || !out_ticket || !out_flags)))
        return OWGS_EINVAL;
    if (n == 0) return OWGS_OK;
    for (int32_t i = 0; i < n; ++i)
        if (off[i + 1] < off[i] || off[i] < 0) return c->fail(OWGS_EINVAL, "offsets");
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    const size_t nb = (size_t)(off[n] - off[0]);
    std::vector<int64_t> o((size_t)n + 1);
    for (int32_t i = 0; i <= n; ++i) o[i] = off[i] - off[0];
    HIPCHK(c, c->k_bytes.reserve(nb + 32));
    HIPCHK(c, hipMemsetAsync(c->k_bytes.p + nb, 0, 32, c->stream));
    if (nb) HIPCHK(c, hipMemcpyAsync(c->k_bytes.p, bytes + off[0], nb, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, upload(c->k_off, o.data(), o.size(), c->stream));
    HIPCHK(c, c->k_kind.reserve((size_t)n));
    HIPCHK(c, c->k_tick.reserve((size_t)n));
    HIPCHK(c, c->k_oflags.reserve((size_t)n));
    HIPCHK(c, c->k_act.reserve((size_t)n));
    int rc = owgs_process_acks_device(c, n, c->k_bytes.p, c->k_off.p, c->k_kind.p, c->k_act.p, c->k_tick.p,
                                      c->k_oflags.p, nullptr);
    if (rc) return rc;
    HIPCHK(c, hipMemcpy(out_kind, c->k_kind.p, (size_t)n, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(out_invoker, c->k_act.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(out_ticket, c->k_tick.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(out_flags, c->k_oflags.p, (size_t)n, hipMemcpyDeviceToHost));
    return OWGS_OK;
}

int owgs_complete_activations(owgs_ctx* c, int32_t n, const char* aid32, const int32_t* invoker, const uint8_t* flags,
                              uint8_t* out_kind, int32_t* out_ticket, uint8_t* out_flags) {
    if (!c || n < 0 || (n > 0 && (!aid32 || !invoker || !flags || !out_kind || !out_ticket || !out_flags)))
        return OWGS_EINVAL;
    if (n == 0) return OWGS_OK;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    HIPCHK(c, upload(c->k_aid, aid32, (size_t)n * 32, c->stream));
    HIPCHK(c, upload(c->k_cfl, flags, (size_t)n, c->stream));
    HIPCHK(c, upload(c->k_act, invoker, (size_t)n, c->stream));
    HIPCHK(c, c->k_key.reserve((size_t)n));
    HIPCHK(c, c->k_info.reserve((size_t)n));
    HIPCHK(c, c->k_inst.reserve((size_t)n));
    HIPCHK(c, c->k_kind.reserve((size_t)n));
    HIPCHK(c, c->k_tick.reserve((size_t)n));
    HIPCHK(c, c->k_oflags.reserve((size_t)n));
    HIPCHK(c, owgs_launch_aid_decode(c->k_aid.p, n, c->k_cfl.p, c->k_key.p, c->k_info.p, c->k_inst.p, c->k_act.p,
                                     c->stream));
    int rc = ack_complete(c, n, c->k_kind.p, c->k_tick.p, c->k_oflags.p, c->stream);
    if (rc) return rc;
    HIPCHK(c, hipMemcpy(out_kind, c->k_kind.p, (size_t)n, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(out_ticket, c->k_tick.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(out_flags, c->k_oflags.p, (size_t)n, hipMemcpyDeviceToHost));
    return OWGS_OK;
}

// ------------------------------------------------------------------------------------------ health supervision
// grow a persistent per-invoker array to cap entries, keeping the first `keep`
template <class T>
static hipError_t grow_keep(DevBuf<T>& d, size_t cap, size_t keep, hipStream_t st) {
    DevBuf<T> nb;
    hipError_t e = nb.reserve(cap);
    if (e != hipSuccess) return e;
    if (keep && d.p) {
        e = hipMemcpyAsync(nb.p, d.p, keep * sizeof(T), hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) {
            nb.release();
            return e;
        }
        e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            nb.release();
            return e;
        }
    }
    d.release();
    d = nb;
    nb.p = nullptr;
    nb.n = 0;
    return hipSuccess;
}

int owgs_health_events(owgs_ctx* c, int32_t n, const int32_t* invoker, const uint8_t* kind, const int64_t* t_ms,
                       const int64_t* user_memory_bytes, int64_t now_ms, int32_t apply) {
    if (!c || n < 0 || (n > 0 && (!invoker || !kind || !t_ms || !user_memory_bytes))) return OWGS_EINVAL;
    // argument contract (mailbox order with a clock): validated before any state changes
    int64_t prev = c->h_now;
    int32_t max_id = -1, max_ping = -1;
    for (int32_t e = 0; e < n; ++e) {
        if (kind[e] > OWGS_EV_STATE_TIMEOUT || invoker[e] < 0 || invoker[e] >= OWGS_HEALTH_MAX_ID || t_ms[e] < prev ||
            t_ms[e] >= (1LL << 60))
            return c->fail(OWGS_EINVAL, "health event: kind > 4, invoker outside [0, 2^24), time before the previous "
                                        "one or outside [0, 2^60)");
        prev = t_ms[e];
        max_id = std::max(max_id, invoker[e]);
        if (kind[e] == OWGS_EV_PING) max_ping = std::max(max_ping, invoker[e]);
    }
    if (now_ms < prev || now_ms < 0 || now_ms >= (1LL << 60))
        return c->fail(OWGS_EINVAL, "health batch: now before its last event or outside [0, 2^60)");
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    hipStream_t st = c->stream;
    const int32_t old_size = c->h_size;
    const int32_t new_size = std::max(old_size, max_ping + 1);
    if (new_size > c->h_cap) {
        int32_t cap = c->h_cap ? c->h_cap : 1024;
        while (cap < new_size) cap *= 2;
        const size_t keep = (size_t)c->h_cap;
        HIPCHK(c, grow_keep(c->h_st, cap, keep, st));
        HIPCHK(c, grow_keep(c->h_ring, cap, keep, st));
        HIPCHK(c, grow_keep(c->h_last, cap, keep, st));
        HIPCHK(c, grow_keep(c->h_tick, cap, keep, st));
        HIPCHK(c, grow_keep(c->h_mem, cap, keep, st));
        HIPCHK(c, grow_keep(c->h_tests, cap, keep, st));
        HIPCHK(c, owgs_launch_health_init(c->h_st.p, c->h_ring.p, c->h_last.p, c->h_tick.p, c->h_mem.p, c->h_tests.p,
                                          c->h_cap, cap, st));
        c->h_cap = cap;
    }
    HIPCHK(c, upload(c->he_inv, invoker, (size_t)n, st));
    HIPCHK(c, upload(c->he_kind, kind, (size_t)n, st));
    HIPCHK(c, upload(c->he_t, t_ms, (size_t)n, st));
    HIPCHK(c, upload(c->he_mem, user_memory_bytes, (size_t)n, st));
    int32_t bits = 1;
    while (bits < 31 && (max_id >> bits) != 0) ++bits;
    const size_t tb = n ? owgs_health_sort_bytes(n, bits) : 0;
    HIPCHK(c, c->he_temp.reserve(tb));
    HIPCHK(c, c->he_key.reserve((size_t)n));
    HIPCHK(c, c->he_idx0.reserve((size_t)n));
    HIPCHK(c, c->he_idx1.reserve((size_t)n));
    HIPCHK(c, c->he_packed.reserve((size_t)n));
    HIPCHK(c, c->he_beg.reserve((size_t)new_size));
    HIPCHK(c, c->he_end.reserve((size_t)new_size));
    HIPCHK(c, c->he_reg.reserve((size_t)new_size));
    HIPCHK(c, c->he_pad.reserve((size_t)new_size));
    HIPCHK(c, owgs_launch_health_batch(c->he_inv.p, c->he_kind.p, c->he_t.p, c->he_mem.p, n, bits, c->he_temp.p, tb,
                                       c->he_key.p, c->he_idx0.p, c->he_idx1.p, c->he_packed.p, c->he_beg.p,
                                       c->he_end.p, c->he_reg.p,
                                       c->he_pad.p, c->h_st.p, c->h_ring.p, c->h_last.p, c->h_tick.p, c->h_mem.p,
                                       c->h_tests.p, old_size, new_size, now_ms, st));
    HIPCHK(c, hipStreamSynchronize(st));
    c->h_size = new_size;
    c->h_now = now_ms;
    if (!apply) return OWGS_OK;
    // CurrentInvokerPoolState -> monitor -> updateInvokers (SCPB:226-227): ids are the positions (InvokerPool keeps
    // status(i).id.toInt == i, ISUP:186-191)
    std::vector<int32_t> ids(new_size);
    std::vector<int64_t> mem(new_size);
    std::vector<uint8_t> sts(new_size);
    int rc = owgs_health_read(c, new_size, nullptr, sts.data(), mem.data(), nullptr, nullptr, nullptr);
    if (rc) return rc;
    for (int32_t i = 0; i < new_size; ++i) ids[i] = i;
    return owgs_update_invokers(c, new_size, ids.data(), mem.data(), sts.data());
}

int owgs_health_read(owgs_ctx* c, int32_t cap, int32_t* n, uint8_t* status, int64_t* user_memory_bytes,
                     int32_t* test_actions, uint32_t* ring, int64_t* next_tick) {
    if (!c || cap < 0) return OWGS_EINVAL;
    if (n) *n = c->h_size;
    const int32_t m = c->h_size;
    if (m == 0) return OWGS_OK;
    if (!status && !user_memory_bytes && !test_actions && !ring && !next_tick) return OWGS_OK;  // size query
    if (cap < m) return c->fail(OWGS_ERANGE, "health read: capacity below the status vector size");
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    hipStream_t st = c->stream;
    if (status) HIPCHK(c, hipMemcpyAsync(status, c->h_st.p, (size_t)m, hipMemcpyDeviceToHost, st));
    if (user_memory_bytes)
        HIPCHK(c, hipMemcpyAsync(user_memory_bytes, c->h_mem.p, (size_t)m * 8, hipMemcpyDeviceToHost, st));
    if (test_actions) HIPCHK(c, hipMemcpyAsync(test_actions, c->h_tests.p, (size_t)m * 4, hipMemcpyDeviceToHost, st));
    if (ring) HIPCHK(c, hipMemcpyAsync(ring, c->h_ring.p, (size_t)m * 4, hipMemcpyDeviceToHost, st));
    if (next_tick) HIPCHK(c, hipMemcpyAsync(next_tick, c->h_tick.p, (size_t)m * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (status)  // an entry without an actor (padToIndexed) is Offline
        for (int32_t i = 0; i < m; ++i)
            if (status[i] > OWGS_OFFLINE) status[i] = OWGS_OFFLINE;
    if (next_tick)
        for (int32_t i = 0; i < m; ++i)
            if (next_tick[i] == INT64_MAX) next_tick[i] = -1;
    return OWGS_OK;
}

// ------------------------------------------------------------------------------------------ ActivationMessage output
int owgs_register_templates(owgs_ctx* c, int32_t n, const char* a_bytes, const int64_t* a_off, const char* b_bytes,
                            const int64_t* b_off, int32_t* out_first_id) {
    if (!c || n < 0 || (n > 0 && (!a_bytes || !a_off || !b_bytes || !b_off))) return OWGS_EINVAL;
    for (int32_t i = 0; i < n; ++i)
        if (a_off[i + 1] < a_off[i] || b_off[i + 1] < b_off[i] || a_off[0] < 0 || b_off[0] < 0)
            return c->fail(OWGS_EINVAL, "template offsets must be non-decreasing");
    if ((int64_t)c->ta_off.size() - 1 + n > INT32_MAX) return c->fail(OWGS_ERANGE, "too many templates");
    if (out_first_id) *out_first_id = (int32_t)c->ta_off.size() - 1;
    for (int32_t i = 0; i < n; ++i) {
        c->ta.insert(c->ta.end(), a_bytes + a_off[i], a_bytes + a_off[i + 1]);
        c->ta_off.push_back((int64_t)c->ta.size());
        c->tb.insert(c->tb.end(), b_bytes + b_off[i], b_bytes + b_off[i + 1]);
        c->tb_off.push_back((int64_t)c->tb.size());
    }
    c->tmpl_dirty = true;
    return OWGS_OK;
}

int owgs_set_root_controller(owgs_ctx* c, const char* json, int32_t len) {
    if (!c || len < 0 || (len > 0 && !json)) return OWGS_EINVAL;
    c->rci.assign(json, json + len);
    c->tmpl_dirty = true;
    return OWGS_OK;
}

static int msg_templates_upload(owgs_ctx* c, hipStream_t st) {
    if (!c->tmpl_dirty) return OWGS_OK;
    HIPCHK(c, upload(c->m_ta, c->ta.data(), c->ta.size(), st));
    HIPCHK(c, upload(c->m_tb, c->tb.data(), c->tb.size(), st));
    HIPCHK(c, upload(c->m_ta_off, c->ta_off.data(), c->ta_off.size(), st));
    HIPCHK(c, upload(c->m_tb_off, c->tb_off.data(), c->tb_off.size(), st));
    HIPCHK(c, upload(c->m_rci, c->rci.data(), c->rci.size(), st));
    HIPCHK(c, hipStreamSynchronize(st));
    c->tmpl_dirty = false;
    return OWGS_OK;
}

// plan + write with device pointers; host-visible *total / *m
static int msg_run(owgs_ctx* c, OwgsMsgArgs& A, int32_t n_topics, hipStream_t st, int64_t* total, int32_t* m) {
    int rc = msg_templates_upload(c, st);
    if (rc) return rc;
    const int32_t n = A.n;
    A.ta = c->m_ta.p;
    A.ta_off = c->m_ta_off.p;
    A.tb = c->m_tb.p;
    A.tb_off = c->m_tb_off.p;
    A.n_templates = (int32_t)c->ta_off.size() - 1;
    A.rci = c->m_rci.p;
    A.rci_len = (int32_t)c->rci.size();
    A.n_topics = n_topics;
    int32_t bits = 1;
    while (bits < 31 && ((int64_t)n_topics >> bits) != 0) ++bits;
    HIPCHK(c, c->m_key.reserve((size_t)n));
    HIPCHK(c, c->m_key_sorted.reserve((size_t)n));
    HIPCHK(c, c->m_len.reserve((size_t)n));
    HIPCHK(c, c->m_len_sorted.reserve((size_t)n + 1));
    HIPCHK(c, c->m_iota.reserve((size_t)n));
    HIPCHK(c, c->m_cnt.reserve((size_t)n_topics + 1));
    HIPCHK(c, c->m_bad.reserve(1));
    const size_t tb = owgs_msg_scratch_bytes(n, n_topics, bits);
    HIPCHK(c, c->m_temp.reserve(tb));
    A.key = c->m_key.p;
    A.len = c->m_len.p;
    A.bad = c->m_bad.p;
    HIPCHK(c, hipMemsetAsync(c->m_bad.p, 0, 4, st));
    HIPCHK(c, owgs_launch_msg_plan(&A, bits, c->m_temp.p, tb, c->m_key_sorted.p, c->m_iota.p, c->m_len_sorted.p,
                                   c->m_cnt.p, st));
    HIPCHK(c, owgs_launch_msg_write(&A, st));
    int32_t bad = 0, mm = 0;
    int64_t tot = 0;
    HIPCHK(c, hipMemcpyAsync(&bad, c->m_bad.p, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(&mm, A.topic_start + n_topics, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(&tot, A.out_off + n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (total) *total = tot;
    if (m) *m = mm;
    if (bad & 1) return c->fail(OWGS_EINVAL, "serialize: invoker >= n_topics or unknown template");
    if (bad & 2) return c->fail(OWGS_EINVAL, "serialize: transaction id is not valid UTF-8");
    if (bad & 4) return c->fail(OWGS_ERANGE, "serialize: output capacity below the batch's bytes (see *total)");
    return OWGS_OK;
}

static bool msg_batch_ok(const owgs_msg_batch* b, int32_t n_topics) {
    if (!b || b->n < 0 || n_topics < 0 || n_topics >= INT32_MAX) return false;
    if (b->n == 0) return true;
    return b->invoker && b->tmpl && b->aid && b->tid_off && b->tid_start && b->flags;
}

int owgs_serialize_activations(owgs_ctx* c, const owgs_msg_batch* b, int32_t n_topics, char* out, int64_t cap,
                               int64_t* out_off, int32_t* out_order, int32_t* topic_start, int64_t* total,
                               int32_t* m) {
    if (!c || !msg_batch_ok(b, n_topics) || cap < 0 || !out_off || !topic_start || (b->n > 0 && !out_order) ||
        (cap > 0 && !out))
        return OWGS_EINVAL;
    const int32_t n = b->n;
    if (n > 0 && b->tid_off[n] > b->tid_off[0] && !b->tid)
        return c->fail(OWGS_EINVAL, "serialize: transaction id bytes missing");
    bool need_c = false, need_r = false, need_x = false;
    for (int32_t i = 0; i < n; ++i) {
        need_c |= (b->flags[i] & OWGS_MSG_HAS_CONTENT) != 0;
        need_x |= (b->flags[i] & OWGS_MSG_HAS_CAUSE) != 0;
        need_r |= (b->flags[i] & OWGS_MSG_HAS_TRACE) != 0;
    }
    if ((need_c && (!b->content || !b->content_off)) || (need_x && !b->cause) || (need_r && (!b->trace || !b->trace_off)))
        return c->fail(OWGS_EINVAL, "serialize: a flag asks for content / cause / traceContext that is missing");
    for (int32_t i = 0; i < n; ++i)
        if (b->tid_off[i + 1] < b->tid_off[i] || (need_c && b->content_off[i + 1] < b->content_off[i]) ||
            (need_r && b->trace_off[i + 1] < b->trace_off[i]))
            return c->fail(OWGS_EINVAL, "serialize: offsets must be non-decreasing");
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, c->stream);
        if (ro_) return ro_;
    }
    hipStream_t st = c->stream;
    const int64_t tid0 = n ? b->tid_off[0] : 0, tidn = n ? b->tid_off[n] : 0;
    HIPCHK(c, upload(c->m_inv, b->invoker, (size_t)n, st));
    HIPCHK(c, upload(c->m_tmpl, b->tmpl, (size_t)n, st));
    HIPCHK(c, upload(c->m_aid, (const ulonglong2*)b->aid, (size_t)n, st));
    HIPCHK(c, upload(c->m_tid, b->tid + tid0, (size_t)(tidn - tid0), st));
    std::vector<int64_t> off((size_t)n + 1);
    for (int32_t i = 0; i <= n; ++i) off[i] = n ? b->tid_off[i] - tid0 : 0;
    HIPCHK(c, upload(c->m_tid_off, off.data(), off.size(), st));
    HIPCHK(c, upload(c->m_tid_start, b->tid_start, (size_t)n, st));
    HIPCHK(c, upload(c->m_flags, b->flags, (size_t)n, st));
    std::vector<int64_t> coff((size_t)n + 1, 0), roff((size_t)n + 1, 0);
    if (need_c) {
        for (int32_t i = 0; i <= n; ++i) coff[i] = b->content_off[i] - b->content_off[0];
        HIPCHK(c, upload(c->m_content, b->content + b->content_off[0], (size_t)coff[n], st));
    }
    if (need_r) {
        for (int32_t i = 0; i <= n; ++i) roff[i] = b->trace_off[i] - b->trace_off[0];
        HIPCHK(c, upload(c->m_trace, b->trace + b->trace_off[0], (size_t)roff[n], st));
    }
    HIPCHK(c, upload(c->m_content_off, coff.data(), coff.size(), st));
    HIPCHK(c, upload(c->m_trace_off, roff.data(), roff.size(), st));
    if (need_x) HIPCHK(c, upload(c->m_cause, (const ulonglong2*)b->cause, (size_t)n, st));
    else HIPCHK(c, c->m_cause.reserve(1));
    HIPCHK(c, c->m_content.reserve(1));
    HIPCHK(c, c->m_trace.reserve(1));
    HIPCHK(c, c->m_order.reserve((size_t)n));
    HIPCHK(c, c->m_out_off.reserve((size_t)n + 1));
    HIPCHK(c, c->m_topic.reserve((size_t)n_topics + 1));
    HIPCHK(c, c->m_out.reserve((size_t)std::max<int64_t>(cap, 1)));
    OwgsMsgArgs A{};
    A.n = n;
    A.invoker = c->m_inv.p;
    A.tmpl = c->m_tmpl.p;
    A.aid = c->m_aid.p;
    A.tid = c->m_tid.p;
    A.tid_off = c->m_tid_off.p;
    A.tid_start = c->m_tid_start.p;
    A.flags = c->m_flags.p;
    A.content = c->m_content.p;
    A.content_off = c->m_content_off.p;
    A.cause = c->m_cause.p;
    A.trace = c->m_trace.p;
    A.trace_off = c->m_trace_off.p;
    A.order = c->m_order.p;
    A.out_off = c->m_out_off.p;
    A.topic_start = c->m_topic.p;
    A.out = c->m_out.p;
    A.cap = cap;
    int64_t tot = 0;
    int32_t mm = 0;
    int rc = msg_run(c, A, n_topics, st, &tot, &mm);
    if (total) *total = tot;
    if (m) *m = mm;
    if (rc) return rc;
    if (tot) HIPCHK(c, hipMemcpyAsync(out, c->m_out.p, (size_t)tot, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(out_off, c->m_out_off.p, (size_t)(mm + 1) * 8, hipMemcpyDeviceToHost, st));
    if (mm) HIPCHK(c, hipMemcpyAsync(out_order, c->m_order.p, (size_t)mm * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(topic_start, c->m_topic.p, (size_t)(n_topics + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    return OWGS_OK;
}

int owgs_serialize_activations_device(owgs_ctx* c, const owgs_msg_batch* b, int32_t n_topics, char* out,
                                      int64_t cap, int64_t* out_off, int32_t* out_order, int32_t* topic_start,
                                      int64_t* total, int32_t* m, void* stream) {
    if (!c || !msg_batch_ok(b, n_topics) || cap < 0 || !out_off || !topic_start || (b->n > 0 && !out_order) ||
        (cap > 0 && !out) || (b->n > 0 && (!b->content_off || !b->trace_off)))
        return OWGS_EINVAL;
    OWGS_ENTER(c);
    {
        const int ro_ = order_on(c, stream ? (hipStream_t)stream : c->stream);
        if (ro_) return ro_;
    }
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(c, c->m_content.reserve(1));
    HIPCHK(c, c->m_trace.reserve(1));
    HIPCHK(c, c->m_cause.reserve(1));
    OwgsMsgArgs A{};
    A.n = b->n;
    A.invoker = b->invoker;
    A.tmpl = b->tmpl;
    A.aid = (const ulonglong2*)b->aid;
    A.tid = b->tid;
    A.tid_off = b->tid_off;
    A.tid_start = b->tid_start;
    A.flags = b->flags;
    A.content = b->content ? b->content : c->m_content.p;
    A.content_off = b->content_off;
    A.cause = b->cause ? (const ulonglong2*)b->cause : c->m_cause.p;
    A.trace = b->trace ? b->trace : c->m_trace.p;
    A.trace_off = b->trace_off;
    A.order = out_order;
    A.out_off = out_off;
    A.topic_start = topic_start;
    A.out = out;
    A.cap = cap;
    return msg_run(c, A, n_topics, st, total, m);
}

int owgs_resident_stats(owgs_ctx* c, int64_t* out, int32_t cap) {
    if (!c || cap < 0 || (cap > 0 && !out)) return OWGS_EINVAL;
    const int64_t v[5] = {c->res_n_calls, c->res_n_launches, c->res_n_bails, c->res_n_chained, c->res_alive ? 1 : 0};
    for (int32_t i = 0; i < cap && i < 5; ++i) out[i] = v[i];
    for (int32_t i = 5; i < cap && i < 5 + OWGS_RES_NPROF; ++i) out[i] = c->res_prof[i - 5];
    if (cap > 5 + OWGS_RES_NPROF) out[5 + OWGS_RES_NPROF] = c->last_call_ns;
    // the last replay in stream mode: its counters, summed over the launch (a synchronisation: diagnostics)
    if (cap > 6 + OWGS_RES_NPROF) {
        out[6 + OWGS_RES_NPROF] = c->spec_last ? 1 : 0;
        unsigned long long v[OWGS_RES_NPROF] = {};
        if (c->spec_last && c->d_spec_stats.p) {
            (void)hipSetDevice(c->cfg.device);
            const int ro_ = order_on(c, c->stream);  // (after the stream-mode replay; a live shim engine is not waited for)
            if (ro_) return ro_;
            HIPCHK(c, hipMemcpyAsync(v, c->d_spec_stats.p, sizeof(v), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
        }
        for (int32_t i = 0; i < OWGS_RES_NPROF && 7 + OWGS_RES_NPROF + i < cap; ++i) out[7 + OWGS_RES_NPROF + i] = (int64_t)v[i];
    }
    if (cap > 7 + 2 * OWGS_RES_NPROF) out[7 + 2 * OWGS_RES_NPROF] = c->res_used_max;
    if (cap > 8 + 2 * OWGS_RES_NPROF) out[8 + 2 * OWGS_RES_NPROF] = c->res_tombs_max;
    if (cap > 9 + 2 * OWGS_RES_NPROF) out[9 + 2 * OWGS_RES_NPROF] = c->res_host_ns[0];
    if (cap > 10 + 2 * OWGS_RES_NPROF) out[10 + 2 * OWGS_RES_NPROF] = c->res_host_ns[1];
    if (cap > 11 + 2 * OWGS_RES_NPROF) out[11 + 2 * OWGS_RES_NPROF] = c->res_n_life;
    if (cap > 12 + 2 * OWGS_RES_NPROF) out[12 + 2 * OWGS_RES_NPROF] = c->res_n_watch_calls;
    return 13 + 2 * OWGS_RES_NPROF;
}

int owgs_engine_ms(owgs_ctx* c, float* ms) {
    if (!c || !ms) return OWGS_EINVAL;
    if (!c->ev_engine_valid) return c->fail(OWGS_ENOENT, "no engine launch yet");
    (void)hipSetDevice(c->cfg.device);  // (counters and events only: the resident engine keeps running)
    HIPCHK(c, hipEventSynchronize(c->ev_engine[1]));
    HIPCHK(c, hipEventElapsedTime(ms, c->ev_engine[0], c->ev_engine[1]));
    return OWGS_OK;
}
