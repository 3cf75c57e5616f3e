// cp_bench.cpp -- TEST/PROFILING ONLY.  Host control-plane cost of the bench workload with no
// device: the same backend the session uses (device rows are just handles; programs are built
// and then dropped).  Reports ns per original per thread; build with -pg for gprof.
//
// usage: cp_bench streams=S n=N step=K [workload keys]
#include "../../tonk_amd/csrc/decoder.h"
#include "../../tonk_amd/csrc/workload.h"
#include "../../tonk_amd/csrc/prof.h"

#include <chrono>
#include <x86intrin.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>
#include <map>
#include <memory>
#include <malloc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>

using namespace tamd;

#ifdef TAMD_PROF
namespace tamd { namespace prof {
thread_local uint64_t cycles[kSlots];
thread_local uint64_t calls[kSlots];
const char* const names[kSlots] = {"enc_add", "enc_encode", "enc_ack", "dec_add_orig", "dec_add_rec", "dec_decode",
    "dec_ack", "dec_is_ready", "gen_matrix", "ge", "elim", "lower_tri", "back_sub", "chain_flush", "sym_merge",
    "prepare_flush", "finish_flush", "release", "enc_dense", "enc_light", "enc_emit", "elim_sums", "elim_pairs",
    "elim_fold", "enc_cauchy", "enc_remove", "elim_start", "lane_read", "lane_dyn", "combine", "fold_merge", "alloc",
    "x1", "x2", "x3", "x4"};
} }
#endif

static int g_stub = 0;
static int g_nobatch = 0;
static int g_pipe = 1;
static bool g_contig = true;  // contig=0: the codecs check run contiguity themselves (rows are allocated in order)
static uint64_t g_step_clock = 1000;  // nobatch=1: single adds only (the runner's fallback path)  // stub=1: encoder calls return at once; stub=2: decoder calls too
struct Null {
    struct RecRef { RecoveryOut out; };
    struct DecRef {};
    Context* ctx;
    Encoder* enc;
    Decoder* dec;
    std::vector<RowId> enc_rows, dec_rows;
    uint64_t instrs = 0;
    // (rows are allocated in order per side: each side's offsets are affine)
    uint32_t pool = 0;  // rows per side; original i uses row i mod pool
    uint64_t layout(const std::vector<RowId>& rows, uint32_t index, uint32_t k) const {
        if (index % pool + k > pool) return 0;
        const uint32_t o0 = ctx->rows.offset(rows[0]), stride = ctx->rows.offset(rows[1]) - o0;
        return (uint64_t)(o0 + (index % pool) * stride) << 32 | stride;
    }
    int enc_add(uint32_t index, uint32_t len, uint32_t* col) {
        const uint32_t hb = length_header_bytes(len);
        TAMD_PROF_SCOPE(kEncAdd);
        if (g_stub) { *col = index; return 0; }
        return enc->add(enc_rows[index], hb + len, hb, len, nullptr, col, true);
    }
    bool enc_add_run(uint32_t index, uint32_t k, uint32_t len, uint32_t* col0) {
        if (g_stub || g_nobatch) return false;
        const uint32_t hb = length_header_bytes(len);
        TAMD_PROF_SCOPE(kEncAdd);
        return enc->add_run(&enc_rows[index], k, hb + len, hb, len, true, col0, g_contig ? layout(enc_rows, index, k) : 0);
    }
    bool dec_add_run(uint32_t col0, uint32_t index, uint32_t k, uint32_t len) {
        if (g_stub > 1 || g_nobatch) return false;
        const uint32_t hb = length_header_bytes(len);
        TAMD_PROF_SCOPE(kDecAddOrig);
        return dec->add_run_inorder(col0, &dec_rows[index], k, hb + len, hb, len, true, g_contig ? layout(dec_rows, index, k) : 0);
    }
    int enc_encode(RecRef& r) { TAMD_PROF_SCOPE(kEncEncode); if (g_stub) return 2; return enc->encode(r.out); }
    int enc_ack(const uint8_t* b, uint32_t n, uint32_t* next) { TAMD_PROF_SCOPE(kEncAck); return enc->acknowledge(b, n, next); }
    int enc_is_ready() { return enc->remaining_slots() <= 2 ? (int)kMaxPacketsReached : 0; }
    int dec_add_original(uint32_t col, uint32_t index, uint32_t len) {
        const uint32_t hb = length_header_bytes(len);
        TAMD_PROF_SCOPE(kDecAddOrig);
        if (g_stub > 1) return 0;
        bool took = false;
        const int r = dec->add_original(col, dec_rows[index], hb + len, hb, len, nullptr, &took, true);
        return r;
    }
    void recovery_lost(const RecRef& r) { ctx->rows.free_deferred(r.out.row); }
    int dec_add_recovery(const RecRef& r) {
        uint8_t tail[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint32_t tl = r.out.total() < 8 ? r.out.total() : 8;
        memcpy(tail + tl - r.out.footer_len, r.out.footer, r.out.footer_len);
        TAMD_PROF_SCOPE(kDecAddRec);
        bool took = false;
        const int rc = dec->add_recovery(r.out.row, r.out.total(), tail, nullptr, &took);
        if (!took) ctx->rows.free_deferred(r.out.row);
        return rc;
    }
    int dec_is_ready() { TAMD_PROF_SCOPE(kDecIsReady); if (g_stub > 1) return 2; return dec->is_ready(); }
    std::vector<RecoveredPacket*> got;
    int dec_decode(std::vector<uint32_t>& nums, DecRef&) {
        TAMD_PROF_SCOPE(kDecDecode);
        got.clear();
        const int rc = dec->decode(got);
        if (rc == 0) for (auto* p : got) nums.push_back(p->packet_num);
        return rc;
    }
    int dec_ack(uint8_t* b, uint32_t l, uint32_t* u) { TAMD_PROF_SCOPE(kDecAck); return dec->ack(b, l, u); }
    void stats(uint64_t e[9], uint64_t d[11]) { enc->stats(e, 9); dec->stats(d, 11); }
    void set_time(uint64_t) {}
    int enc_retransmit(uint32_t*, uint32_t*, const uint8_t**) { return 2; }
};

struct NoTr {
    void on_encode(int, const Null::RecRef&) {}
    void on_decode(int, const std::vector<uint32_t>&, const Null::DecRef&) {}
    void on_ack(int, const uint8_t*, uint32_t, int, uint32_t) {}
    void on_event(char, int, uint32_t, uint32_t) {}
    void on_stats(const uint64_t*, const uint64_t*) {}
    void on_retransmit(int, uint32_t, uint32_t, uint64_t) {}
};

// Poor man's sampling profiler (no perf in the container): SIGPROF every 100 us of CPU time
// records the interrupted PC; `sample=FILE` writes them for addr2line.
static uint64_t g_samples[1 << 20], g_callers[1 << 20], g_callers2[1 << 20];
static volatile size_t g_nsamples = 0;
static volatile int g_sampling = 0;  // samples are kept only inside timed loops
static void on_prof(int, siginfo_t*, void* uc) {
    const size_t n = g_nsamples;
    if (g_sampling && n < (1u << 20)) {
        g_samples[n] = (uint64_t)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP];
        // top of stack: the return address when the sample lands in a frameless leaf (memmove)
        g_callers[n] = *(const uint64_t*)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RSP];
        // and the frame-pointer parent of that caller (builds with -fno-omit-frame-pointer)
        const uint64_t* fp = (const uint64_t*)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RBP];
        const uint64_t sp = (uint64_t)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RSP];
        g_callers2[n] = ((uint64_t)fp >= sp && (uint64_t)fp < sp + (1u << 20) && ((uint64_t)fp & 7) == 0) ? fp[1] : 0;
        g_nsamples = n + 1;
    }
}

// Rows read per program by instruction kind: ACC/ACC3 rows and ACCR runs by mode (CAUCHY split
// into plain -- encoder windows -- and scaled -- decoder run terms), in row loads and bytes.
static void dump_reads(Context& ctx) {
    const auto& ins = ctx.pb.instrs();
    const char* names[8] = {"acc", "lane3", "cauchy", "const", "multi", "dense", "cauchy_scaled", "acc3"};
    uint64_t rows[8] = {0}, bytes[8] = {0};
    std::map<uint32_t, uint32_t> dense_rows;  // packet row -> DENSE runs reading it
    for (size_t k = 0; k < ins.size(); ++k) {
        const uint32_t kind = ins[k].w0 & 0xff;
        int m = -1;
        uint64_t n = 1;
        if (kind == TAMD_I_ACC) m = 0;
        else if (kind == TAMD_I_ACC3) m = 7;
        else if (kind == TAMD_I_ACCR) {
            const uint32_t mode = (ins[k].w0 >> 8) & 0xff;
            m = mode == TAMD_R_CAUCHY && (ins[k].w0 >> 24) > 1 ? 6 : (int)mode;
            n = ins[k].cap;
        }
        if (m < 0 || m > 7) continue;
        if (m == TAMD_R_DENSE)
            for (uint64_t j = 0; j < n; ++j) dense_rows[ins[k].row + j * ins[k + 1].row]++;
        rows[m] += n;
        bytes[m] += n * ins[k].len;
    }
    for (int m = 0; m < 8; ++m)
        if (rows[m]) fprintf(stderr, "reads %-14s rows %8llu  MB %8.2f\n", names[m], (unsigned long long)rows[m], bytes[m] / 1e6);
    // scaled Cauchy runs (decoder elimination): rows read per op vs distinct rows per op
    {
        uint64_t runs = 0, rd = 0, distinct = 0, ops_multi = 0;
        std::map<uint32_t, uint32_t> all;
        const auto& ops = ctx.pb.ops();
        for (const tamd_op& o : ops) {
            std::map<uint32_t, uint32_t> seen;
            uint32_t nr = 0;
            for (uint32_t k = o.first; k < o.first + o.count; ++k) {
                const uint32_t kind = ins[k].w0 & 0xff;
                if (kind != TAMD_I_ACCR) continue;
                const uint32_t mode = (ins[k].w0 >> 8) & 0xff;
                if (mode != TAMD_R_CAUCHY || (ins[k].w0 >> 24) <= 1) continue;
                ++nr;
                for (uint32_t j = 0; j < ins[k].cap; ++j) seen[ins[k].row + j * ins[k + 1].row]++, all[ins[k].row + j * ins[k + 1].row]++;
                rd += ins[k].cap;
            }
            runs += nr;
            distinct += seen.size();
            ops_multi += nr > 1;
        }
        fprintf(stderr, "scaled cauchy: runs %llu rows %llu distinct-per-op %llu distinct %zu ops with >1 run %llu\n",
                (unsigned long long)runs, (unsigned long long)rd, (unsigned long long)distinct, all.size(),
                (unsigned long long)ops_multi);
        // every row any op reads, against the distinct rows
        std::map<uint32_t, uint32_t> every;
        uint64_t tot = 0;
        for (size_t k = 0; k < ins.size(); ++k) {
            const uint32_t kind = ins[k].w0 & 0xff;
            if (kind == TAMD_I_ACC || kind == TAMD_I_ACC3) { every[ins[k].row]++; ++tot; }
            else if (kind == TAMD_I_ACCR)
                for (uint32_t j = 0; j < ins[k].cap; ++j) { every[ins[k].row + j * ins[k + 1].row]++; ++tot; }
        }
        fprintf(stderr, "all reads %llu distinct rows %zu\n", (unsigned long long)tot, every.size());
        // rows read by each run mode, and by the encoder's MULTI and DENSE runs together
        std::map<uint32_t, uint32_t> by_mode[8];
        for (size_t k = 0; k < ins.size(); ++k)
            if ((ins[k].w0 & 0xff) == TAMD_I_ACCR) {
                const uint32_t mode = (ins[k].w0 >> 8) & 7;
                for (uint32_t j = 0; j < ins[k].cap; ++j) by_mode[mode][ins[k].row + j * ins[k + 1].row]++;
            }
        size_t both = 0, md_reads = 0;
        std::map<uint32_t, uint32_t> md;
        for (int m : {TAMD_R_MULTI, TAMD_R_DENSE, TAMD_R_CAUCHY, TAMD_R_CONST})
            for (const auto& kv : by_mode[m]) { md[kv.first] += kv.second; md_reads += kv.second; }
        for (const auto& kv : by_mode[TAMD_R_MULTI]) both += by_mode[TAMD_R_DENSE].count(kv.first);
        fprintf(stderr, "encoder-side runs (multi+dense+cauchy+const): reads %zu distinct %zu; rows in both multi and dense %zu\n",
                md_reads, md.size(), both);
    }
    // rows read by op kind: recovery rows (a STORE with a footer), lane scans (STOREC / ACC3 /
    // LANE3), other (decoder rows, partial sums, temps)
    {
        uint64_t by[3] = {0, 0, 0}, nops[3] = {0, 0, 0};
        for (const tamd_op& o : ctx.pb.ops()) {
            uint64_t rd = 0;
            int kind = 2;
            for (uint32_t k = o.first; k < o.first + o.count; ++k) {
                const uint32_t w = ins[k].w0, kk = w & 0xff;
                if (kk == TAMD_I_ACC || kk == TAMD_I_ACC3) ++rd;
                else if (kk == TAMD_I_ACCR) {
                    rd += ins[k].cap;
                    if (((w >> 8) & 0xff) == TAMD_R_LANE3) kind = 1;
                }
                if (kk == TAMD_I_STOREC || kk == TAMD_I_ACC3) kind = 1;
                if (kk == TAMD_I_STORE && ((w >> 8) & 0xff) && kind != 1) kind = 0;
            }
            by[kind] += rd;
            nops[kind]++;
        }
        fprintf(stderr, "reads by op kind: recovery rows %llu (%llu ops), lane scans %llu (%llu ops), other %llu (%llu ops)\n",
                (unsigned long long)by[0], (unsigned long long)nops[0], (unsigned long long)by[1], (unsigned long long)nops[1],
                (unsigned long long)by[2], (unsigned long long)nops[2]);
    }
    uint64_t hist[5] = {0, 0, 0, 0, 0};
    for (const auto& kv : dense_rows) hist[kv.second < 4 ? kv.second : 4]++;
    fprintf(stderr, "dense: %zu distinct packet rows; read by 1/2/3/4+ runs: %llu %llu %llu %llu\n", dense_rows.size(),
            (unsigned long long)hist[1], (unsigned long long)hist[2], (unsigned long long)hist[3], (unsigned long long)hist[4]);
}

static void dump_levels(Context& ctx) {
            for (size_t b = 0; b < ctx.pb.level_ops().size(); ++b)
                fprintf(stderr, "bucket %zu (level %zu class %zu): ops %u items %u\n", b, b / TAMD_COST_CLASSES, b % TAMD_COST_CLASSES,
                        ctx.pb.level_ops()[b], ctx.pb.level_items()[b]);
            // per bucket: row loads per op (ACC/ACC3 = 1, ACCR = count), histogram and max
            const auto& ops = ctx.pb.ops();
            const auto& ins = ctx.pb.instrs();
            const auto& lv = ctx.pb.op_levels();
            for (size_t b = 0; b < ctx.pb.level_ops().size(); ++b) {
                uint64_t hist[8] = {0}, tot = 0, mx = 0, n = 0, instr = 0;
                for (size_t i = 0; i < ops.size(); ++i) {
                    if (lv[i] != b) continue;
                    uint64_t loads = 0;
                    for (uint32_t k = ops[i].first; k < ops[i].first + ops[i].count; ++k) {
                        const uint32_t kind = ins[k].w0 & 0xff;
                        if (kind == TAMD_I_ACC || kind == TAMD_I_ACC3) ++loads;
                        else if (kind == TAMD_I_ACCR) loads += ins[k].cap;
                    }
                    int h = 0;
                    while (h < 7 && (1ull << (2 * h + 2)) <= loads) ++h;
                    ++hist[h];
                    tot += loads;
                    instr += ops[i].count;
                    if (loads > mx) mx = loads;
                    ++n;
                }
                if (!n) continue;
                fprintf(stderr, "  bucket %zu: loads/op avg %.1f max %llu instrs/op %.1f  hist(<4,<16,<64,<256,..):", b,
                        (double)tot / n, (unsigned long long)mx, (double)instr / n);
                for (int h = 0; h < 8; ++h) fprintf(stderr, " %llu", (unsigned long long)hist[h]);
                fprintf(stderr, "\n");
                // instruction mix: kind (ACC split by coef==1), ACCR by mode with its row count
                uint64_t kinds[16] = {0}, rrows[4] = {0}, rcount[4] = {0};
                for (size_t i = 0; i < ops.size(); ++i) {
                    if (lv[i] != b) continue;
                    for (uint32_t k = ops[i].first; k < ops[i].first + ops[i].count; ++k) {
                        const uint32_t kind = ins[k].w0 & 0xff;
                        if (kind == TAMD_I_ACC && ((ins[k].w0 >> 8) & 0xff) == 1) ++kinds[15];
                        else ++kinds[kind & 15];
                        if (kind == TAMD_I_ACCR) {
                            const uint32_t m = (ins[k].w0 >> 8) & 3;
                            ++rcount[m];
                            rrows[m] += ins[k].cap;
                        }
                    }
                }
                fprintf(stderr, "    ACC(c!=1) %llu ACC(c=1) %llu ACC3 %llu STORE %llu STOREC %llu CLEAR %llu | "
                        "ACCR lane3 %llu (%.1f rows) cauchy %llu (%.1f) const %llu (%.1f)\n",
                        (unsigned long long)kinds[TAMD_I_ACC], (unsigned long long)kinds[15],
                        (unsigned long long)kinds[TAMD_I_ACC3], (unsigned long long)kinds[TAMD_I_STORE],
                        (unsigned long long)kinds[TAMD_I_STOREC], (unsigned long long)kinds[TAMD_I_CLEAR],
                        (unsigned long long)rcount[1], rcount[1] ? (double)rrows[1] / rcount[1] : 0.0,
                        (unsigned long long)rcount[2], rcount[2] ? (double)rrows[2] / rcount[2] : 0.0,
                        (unsigned long long)rcount[3], rcount[3] ? (double)rrows[3] / rcount[3] : 0.0);
            }
        }

int main(int argc, char** argv) {
    const char* sample_out = nullptr;
    for (int i = 1; i < argc; ++i)
        if (!strncmp(argv[i], "sample=", 7)) sample_out = argv[i] + 7;
    gf_init();
    wl::Params p;
    p.loss_thresh = 42949673;
    p.fec_rate_q16 = 1311;
    p.ack_every = 64;
    uint32_t streams = 8, step = 4096, warm_steps = 0, expand = ~0u, backsub = ~0u, reps = 1;  // warm: untimed, unsampled first steps
    p.n_originals = 4096 * 6;
    for (int i = 1; i < argc; ++i) {
        const char* eq = strchr(argv[i], '=');
        if (!eq) continue;
        std::string k(argv[i], eq - argv[i]);
        if (k == "sample") continue;
        if (k == "stub") { g_stub = atoi(eq + 1); continue; }
        if (k == "nobatch") { g_nobatch = atoi(eq + 1); continue; }
        if (k == "warm") { warm_steps = (uint32_t)atoi(eq + 1); continue; }
        if (k == "expand") { expand = (uint32_t)strtoul(eq + 1, nullptr, 0); continue; }
        if (k == "backsub") { backsub = (uint32_t)strtoul(eq + 1, nullptr, 0); continue; }
        if (k == "pipe") { g_pipe = atoi(eq + 1); continue; }
        if (k == "contig") { g_contig = atoi(eq + 1) != 0; continue; }
        if (k == "reps") { reps = (uint32_t)atoi(eq + 1); continue; }  // level pipelining as the session runs it
        if (k == "prefault") {  // MB of heap faulted in and kept before the run (cold-start studies)
            const size_t mb = (size_t)atoi(eq + 1);
            mallopt(M_MMAP_THRESHOLD, 512 << 20);
            mallopt(M_TRIM_THRESHOLD, 1 << 30);
            void* m = malloc(mb << 20);
            if (m) memset(m, 1, mb << 20);
            free(m);
            continue;
        }
        const unsigned long long v = strtoull(eq + 1, nullptr, 0);
        if (k == "streams") streams = (uint32_t)v;
        else if (k == "n") p.n_originals = (uint32_t)v;
        else if (k == "step") step = (uint32_t)v;
        else if (k == "loss") p.loss_thresh = (uint32_t)v;
        else if (k == "fec") p.fec_rate_q16 = (uint32_t)v;
        else if (k == "ack") p.ack_every = (uint32_t)v;
        else if (k == "ge") p.ge_enable = (uint32_t)v;
        else if (k == "gb") p.gb_thresh = (uint32_t)v;
        else if (k == "bg") p.bg_thresh = (uint32_t)v;
        else if (k == "arq") p.arq_lag = (uint32_t)v;
    }
    // reps=R: the whole run is repeated R times with fresh codecs; every (step, stream) segment
    // is timed (TSC) and the sum over segments of each segment's minimum over the repetitions is
    // reported (segmin_cyc_per_original): a host-load burst inflates one repetition's segment,
    // not all of them.
    std::vector<uint64_t> seg_min;
    std::chrono::steady_clock::time_point t0;
    double c0 = 0;
    uint32_t timed_originals = 0;
    uint64_t instrs = 0, ops = 0, acc_bytes = 0, store_bytes = 0;
    auto cpu_now = []() {
        timespec ts;
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
        return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
    };
    uint32_t last_enc_window = 0;
    for (uint32_t rep = 0; rep < reps; ++rep) {
    // One Context per stream with each side's input rows contiguous, as the session lays them out
    // (tamd_session_generate), and steps of `step` originals per stream.
    std::vector<std::unique_ptr<Context>> ctxs(streams);
    std::vector<std::unique_ptr<Null>> be(streams);
    std::vector<std::unique_ptr<Encoder>> encs(streams);
    std::vector<std::unique_ptr<Decoder>> decs(streams);
    std::vector<wl::Params> ps(streams, p);
    NoTr tr;
    std::vector<std::unique_ptr<wl::Runner<Null, NoTr>>> run(streams);
    for (uint32_t s = 0; s < streams; ++s) {
        ps[s].seed_data = 1000 + s;
        ps[s].seed_loss = 2000 + s;
        ctxs[s].reset(new Context());
        Context& ctx = *ctxs[s];
        ctx.ex.expand_limit = expand;
        ctx.backsub_rows = backsub;
        ctx.dense_split = getenv("TONK_AMD_DENSE_SPLIT") ? (uint32_t)atoi(getenv("TONK_AMD_DENSE_SPLIT"))
                                                        : (streams > 4 ? Encoder::kDenseSplit : 0u);
        ctx.pipeline = g_pipe != 0;
        ctx.rows.init(4ull * std::min<uint32_t>(p.n_originals, 65536) * 1344 + (256u << 20));
        encs[s].reset(new Encoder(&ctx, 1344));
        encs[s]->set_clock(&g_step_clock);  // the session reads the clock once per step
        decs[s].reset(new Decoder(&ctx, 1344));
        be[s].reset(new Null());
        be[s]->ctx = &ctx;
        be[s]->enc = encs[s].get();
        be[s]->dec = decs[s].get();
        // (a pool of 65536 rows per side, as the bench's sessions: long runs fit in memory)
        const uint32_t pool = std::min<uint32_t>(p.n_originals, 65536);
        be[s]->pool = pool;
        for (uint32_t i = 0; i < pool; ++i) be[s]->enc_rows.push_back(ctx.rows.alloc(1302));
        for (uint32_t i = 0; i < pool; ++i) be[s]->dec_rows.push_back(ctx.rows.alloc(1302));
        for (uint32_t i = pool; i < p.n_originals; ++i) be[s]->enc_rows.push_back(be[s]->enc_rows[i - pool]);
        for (uint32_t i = pool; i < p.n_originals; ++i) be[s]->dec_rows.push_back(be[s]->dec_rows[i - pool]);
        run[s].reset(new wl::Runner<Null, NoTr>(ps[s], *be[s], tr));
        run[s]->pregenerate();
    }
    instrs = ops = acc_bytes = store_bytes = 0;
    timed_originals = 0;
    auto start_sampling = [&]() {
        if (!sample_out) return;
        struct sigaction sa;
        memset(&sa, 0, sizeof(sa));
        sa.sa_sigaction = on_prof;
        sa.sa_flags = SA_SIGINFO | SA_RESTART;
        sigaction(SIGPROF, &sa, nullptr);
        itimerval tv;
        tv.it_interval.tv_sec = 0;
        tv.it_interval.tv_usec = 100;
        tv.it_value = tv.it_interval;
        setitimer(ITIMER_PROF, &tv, nullptr);
        g_sampling = 1;
    };
    t0 = std::chrono::steady_clock::now();
    c0 = cpu_now();
    uint32_t step_no = 0;
    if (!warm_steps) start_sampling();
    for (uint32_t done = 0; done < p.n_originals; done += step, ++step_no) {
        if (warm_steps && step_no == warm_steps) {
            t0 = std::chrono::steady_clock::now();
            c0 = cpu_now();
#ifdef TAMD_PROF
            memset(prof::cycles, 0, sizeof(prof::cycles));
            memset(prof::calls, 0, sizeof(prof::calls));
#endif
            start_sampling();
        }
        if (step_no >= warm_steps) timed_originals += (done + step <= p.n_originals ? step : p.n_originals - done);
        for (uint32_t s = 0; s < streams; ++s) {
            Context& ctx = *ctxs[s];
            const uint64_t seg0 = __rdtsc();
            run[s]->advance(step);
            const uint64_t e = ctx.epoch;
            {
                TAMD_PROF_SCOPE(kFlushAll);
                ctx.prepare_flush();
            }
            if (getenv("CP_BENCH_LEVELS") && done == step && s == 0) dump_levels(ctx);
            if (getenv("CP_BENCH_READS") && done == step && s == 0) dump_reads(ctx);
            instrs += ctx.pb.instrs().size();
            ops += ctx.pb.ops().size();
            acc_bytes += ctx.pb.acc_bytes();
            store_bytes += ctx.pb.store_bytes();
            {
                TAMD_PROF_SCOPE(kFinish);
                ctx.finish_flush();
            }
            {
                TAMD_PROF_SCOPE(kRelease);
                ctx.rows.release_up_to(e);
            }
            if (step_no >= warm_steps) {
                const uint64_t c = __rdtsc() - seg0;
                const size_t si = (size_t)(step_no - warm_steps) * streams + s;
                if (seg_min.size() <= si) seg_min.resize(si + 1, ~0ull);
                if (c < seg_min[si]) seg_min[si] = c;
            }
        }
    }
    g_sampling = 0;
    last_enc_window = (unsigned)(kMaxPackets - encs[0]->remaining_slots());
    }  // rep
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double cpu_sec = cpu_now() - c0;
    if (sample_out) {
        itimerval off;
        memset(&off, 0, sizeof(off));
        setitimer(ITIMER_PROF, &off, nullptr);
        FILE* f = fopen(sample_out, "w");
        for (size_t i = 0; i < g_nsamples; ++i) fprintf(f, "%llx\n", (unsigned long long)g_samples[i]);
        fclose(f);
        f = fopen((std::string(sample_out) + ".callers").c_str(), "w");
        for (size_t i = 0; i < g_nsamples; ++i)
            fprintf(f, "%llx %llx %llx\n", (unsigned long long)g_samples[i], (unsigned long long)g_callers[i],
                    (unsigned long long)g_callers2[i]);
        fclose(f);
        // the process's mappings, to resolve samples inside shared libraries
        std::string mp = std::string(sample_out) + ".maps";
        FILE* in = fopen("/proc/self/maps", "r");
        FILE* out = fopen(mp.c_str(), "w");
        char line[512];
        while (in && out && fgets(line, sizeof(line), in)) fputs(line, out);
        if (in) fclose(in);
        if (out) fclose(out);
    }
    if (getenv("CP_BENCH_WIN")) fprintf(stderr, "enc window %u\n", last_enc_window);
    const double n = (double)streams * timed_originals;
    uint64_t segsum = 0;
    for (uint64_t c : seg_min) segsum += c;
    printf("{\"segmin_cyc_per_original\": %.1f, \"cpu_ns_per_original\": %.1f, \"ns_per_original\": %.1f, \"instrs_per_original\": %.2f, \"ops_per_original\": %.3f, "
           "\"acc_bytes_per_original\": %.0f, \"store_bytes_per_original\": %.0f, \"seconds\": %.3f}\n",
           (double)segsum / n, cpu_sec * 1e9 / n, sec * 1e9 / n, instrs / n, ops / n, acc_bytes / n, store_bytes / n, sec);
#ifdef TAMD_PROF
    const double ghz = 1.0 * 0 + 1;
    for (int i = 0; i < prof::kSlots; ++i)
        if (prof::calls[i])
            fprintf(stderr, "%-14s calls/orig %8.4f  cyc/call %10.0f  cyc/orig %8.1f\n", prof::names[i],
                    prof::calls[i] / n, (double)prof::cycles[i] / prof::calls[i], prof::cycles[i] / n * ghz);
#endif
    return 0;
}
