// cp_harness.cpp -- TEST ONLY.  Drives the MI355X engine's host control plane (encoder.cpp,
// decoder.cpp, engine.cpp) through the synthetic workload with NO GPU: the device programs the
// control plane emits are executed by the oracle's CPU interpreter (oracle/siamese_oracle.c)
// over a host copy of the arena, and the run writes the same transcript as
// oracle/golden_gen.cpp does for the reference codec.  Used by tests/test_control_plane.py to
// pin the control plane (every decision and every recovery/recovered byte) on CPU-only hosts.
//
// usage: cp_harness <out.txt> mode=sync|batch batch=K key=value...
#include "../../tonk_amd/csrc/encoder.h"
#include "../../tonk_amd/csrc/decoder.h"
#include "../../tonk_amd/csrc/workload.h"
#include "../../tonk_amd/csrc/transcript.h"
#include "../../tonk_amd/csrc/prof.h"
#include "../../oracle/siamese_oracle.h"

#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>

using namespace tamd;
using namespace tamd::wl;

static uint64_t g_arena_bytes = 512ull << 20;
// dirty=1: the context visits only codecs touched since the last flush (Context::track_dirty,
// as the siamese.h C ABI runs it); every backend call touches its codec like capi.cpp does.
static bool g_dirty = false;
static bool g_nobatch = false;  // nobatch=1: the runner's single-add path only
static int g_ddirect = -1;  // ddirect=0/1: decoder eliminations through the lanes / direct (default: the engine's)
// pipeline=1: the session's pipelined launches (Device::launch_step: level 1 of a program beside
// the next level of every older program in flight) are simulated and every launch is checked for
// hazards (no segment reads or writes a row another writes) before the programs run in order.
static bool g_pipeline = false;
static uint32_t g_expand = ~0u;  // expand=<terms>: the session's expansion limit
static uint32_t g_backsub = ~0u;  // backsub=<unknowns>: back substitution over materialized rows
static uint32_t g_split = 0;      // split=<packets>: the batched session's dense-range split
// ahead=<K>: encode-ahead as the C ABI runs it (capi.cpp): from the second encode in a row (no
// other encoder call between) up to K more encodes run ahead while Encoder::encode_is_quiet, and
// are handed out by the next encode calls; any other encoder call first takes the rest back
// (Encoder::rewind) and frees their rows.  The depth doubles from 1 while they are all used.
static uint32_t g_ahead = 0;
static bool g_short = false;  // short=1: Context::short_scans (the C ABI's lane-sum snapshot levels)
static uint64_t g_rs[9];  // CP_READ_STATS totals
static bool g_contig = false;  // contig=1: originals in rows reserved up front, in order, one range per
                               // side and borrowed by the codecs (the batched session's layout)
static uint32_t g_drain = 0;  // pipelined: complete every in-flight program after every g_drain-th (session record mode: 2)
#include <map>
#include <set>
#include <unordered_map>

#ifdef TAMD_PROF  // (_build/cp_harness_prof: cycles per control-plane phase at exit)
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

struct Harness {
    Params p;
    Context ctx;
    std::vector<uint8_t> arena;
    Encoder* enc = nullptr;
    Decoder* dec = nullptr;
    uint32_t row_bytes = 0;
    bool sync = true;
    uint32_t batch = 0;
    TextSink out;
    uint64_t programs = 0, ops = 0, levels = 0, instrs = 0;
    std::string error;
    // rows read / written per level of a program (pipelined launch checks)
    struct LevelRW { std::set<uint32_t> rd, wr; };
    uint64_t pipelined_pairs = 0;

    std::vector<LevelRW> level_rw() const {
        const auto& ops_v = ctx.pb.ops();
        const auto& lv = ctx.pb.op_levels();
        const auto& in = ctx.pb.instrs();
        std::vector<LevelRW> out(ctx.pb.max_level() + 1);
        for (size_t i = 0; i < ops_v.size(); ++i) {
            LevelRW& r = out[lv[i] / TAMD_COST_CLASSES];
            for (uint32_t k = ops_v[i].first; k < ops_v[i].first + ops_v[i].count; ++k) {
                const uint32_t kind = in[k].w0 & 0xff;
                if (kind == TAMD_I_ACC || kind == TAMD_I_ACC3) r.rd.insert(in[k].row);
                else if (kind == TAMD_I_ACCR)
                    for (uint32_t q = 0; q < in[k].cap; ++q) r.rd.insert(in[k].row + q * in[k + 1].row);
                else if (kind == TAMD_I_STORE || kind == TAMD_I_STOREC) r.wr.insert(in[k].row);
            }
        }
        return out;
    }
    // Every launch runs level 1 of this program beside the next level of each older program
    // still in flight (Device::launch_step).  Each level's dependencies in program order (the
    // last writer of every row it reads or writes, and the readers since, of any program) must
    // have run in an EARLIER launch: same-launch and out-of-order hazards alike, including rows
    // reused after release.
    typedef std::pair<uint64_t, uint32_t> Lv;  // (program epoch, level)
    struct RowHist { Lv w{0, 0}; std::vector<Lv> rd; };
    std::unordered_map<uint32_t, RowHist> hist;
    std::map<Lv, uint64_t> launched_at;
    uint64_t launch_no = 0;
    struct Prog { std::vector<LevelRW> levels; std::vector<std::vector<Lv>> deps; uint32_t next = 1; uint64_t epoch = 0; };
    std::vector<Prog> inflight;
    uint64_t launched = 0;
    void check_pipeline() {
        Prog cur;
        cur.levels = level_rw();
        cur.epoch = ctx.epoch;
        cur.deps.resize(cur.levels.size());
        for (uint32_t d = 1; d < cur.levels.size(); ++d) {
            const Lv me(cur.epoch, d);
            std::set<Lv> dd;
            for (uint32_t x : cur.levels[d].rd) {
                const RowHist& h = hist[x];
                if (h.w.first) dd.insert(h.w);
            }
            for (uint32_t x : cur.levels[d].wr) {
                const RowHist& h = hist[x];
                if (h.w.first) dd.insert(h.w);
                dd.insert(h.rd.begin(), h.rd.end());
            }
            dd.erase(me);
            cur.deps[d].assign(dd.begin(), dd.end());
            for (uint32_t x : cur.levels[d].rd) hist[x].rd.push_back(me);
            for (uint32_t x : cur.levels[d].wr) {
                RowHist& h = hist[x];
                h.w = me;
                h.rd.clear();
            }
        }
        inflight.push_back(std::move(cur));
        pipeline_step();
        // Device::wait / synchronize: the remaining levels launch without a new program
        if (g_drain && ++launched % g_drain == 0)
            while (!inflight.empty()) pipeline_step();
    }
    void pipeline_step() {
        std::vector<Prog*> run;
        for (Prog& p : inflight)
            if (p.next < p.levels.size()) run.push_back(&p);
        for (Prog* p : run)
            for (const Lv& dep : p->deps[p->next]) {
                const auto it = launched_at.find(dep);
                if ((it == launched_at.end() || it->second >= launch_no) && error.empty())
                    error = "pipelined launch " + std::to_string(launch_no) + ": level " + std::to_string(p->next) +
                            " of program " + std::to_string(p->epoch) + " runs before or with level " +
                            std::to_string(dep.second) + " of program " + std::to_string(dep.first) +
                            " it depends on";
            }
        static const bool trace = getenv("CP_TRACE") != nullptr;
        if (trace) {
            fprintf(stderr, "launch %llu:", (unsigned long long)launch_no);
            for (Prog* p : run) fprintf(stderr, " (%llu,%u)", (unsigned long long)p->epoch, p->next);
            fprintf(stderr, "\n");
        }
        for (Prog* p : run) launched_at[Lv(p->epoch, p->next++)] = launch_no;
        ++launch_no;
        if (run.size() > 1) ++pipelined_pairs;
        size_t keep = 0;
        for (size_t k = 0; k < inflight.size(); ++k)
            if (inflight[k].next < inflight[k].levels.size()) {
                if (k != keep) inflight[keep] = std::move(inflight[k]);  // (no self-move: it empties a vector)
                ++keep;
            }
        inflight.resize(keep);
    }
    // Highest epoch whose programs have all run every level (in the simulated launch order).
    uint64_t release_bound(uint64_t done) const {
        uint64_t b = done;
        for (const Prog& p : inflight)
            if (p.epoch <= b) b = p.epoch - 1;
        return b;
    }

    // transcript entries waiting for their rows to be computed
    struct PendEnc { RowId row; uint32_t total; RecoveryMeta meta; size_t pos; };
    struct PendDec { RowId row; uint32_t upper; size_t pos; };
    std::vector<PendEnc> pend_enc;
    std::vector<std::vector<PendDec>> pend_dec;  // per decode line
    std::vector<size_t> pend_dec_pos;
    std::vector<std::string> lines;  // transcript lines, some filled after execution

    explicit Harness(const Params& prm) : p(prm) {
        row_bytes = ((p.payload_max + 4 + 8 + 63) / 64) * 64;
        ctx.rows.init(g_arena_bytes);
        ctx.track_dirty = g_dirty;
        ctx.pipeline = g_pipeline;
        ctx.ex.expand_limit = g_expand;
        ctx.backsub_rows = g_backsub;
        ctx.dense_split = g_split;
        ctx.short_scans = g_short;
        if (g_ddirect >= 0) ctx.direct_elim = g_ddirect != 0;
        arena.assign(g_arena_bytes, 0);
        enc = new Encoder(&ctx, row_bytes);
        dec = new Decoder(&ctx, row_bytes);
        if (g_contig) {
            const uint32_t cap = p.payload_max + 4;
            for (int side = 0; side < 2; ++side)
                for (uint32_t i = 0; i < p.n_originals; ++i) pre[side].push_back(ctx.alloc(cap));
        }
    }
    std::vector<RowId> pre[2];  // contig=1: the originals' rows of the encoder (0) and decoder (1)
    Encoder* E() {
        if (g_dirty) ctx.touch(enc);
        return enc;
    }
    Decoder* D() {
        if (g_dirty) ctx.touch(dec);
        return dec;
    }
    ~Harness() {
        delete enc;
        delete dec;
    }

    uint8_t* at(RowId r) { return arena.data() + (size_t)ctx.rows.offset(r) * TAMD_ROW_UNIT; }

    RowId write_original(uint32_t index, uint32_t len, uint32_t* framed, uint32_t* header, int side = 0) {
        uint8_t hdr[4];
        const uint32_t hb = put_length_header(len, hdr);
        const RowId r = g_contig ? pre[side][index] : ctx.alloc(hb + len);
        if (r == kNoRow) return r;
        uint8_t* d = at(r);
        memset(d, 0, ctx.rows.cap_bytes(r));
        memcpy(d, hdr, hb);
        payload_bytes(p, index, d + hb, len);
        *framed = hb + len;
        *header = hb;
        return r;
    }

    // Within a program the device runs each level's ops together, in no order (levels run in
    // order, which the oracle's level-by-level run checks through the outputs): no row one op of
    // a level writes may be read or written by another op of the same level.
    void check_levels() {
        const auto& ops_v = ctx.pb.ops();
        const auto& lv = ctx.pb.op_levels();
        const auto& in = ctx.pb.instrs();
        std::unordered_map<uint64_t, uint32_t> writer;  // (level, row) -> op that writes it
        auto bad = [&](size_t i, uint32_t l, uint32_t x, uint32_t other) {
            if (error.empty())
                error = "program " + std::to_string(programs) + ": ops " + std::to_string(other) + " and " +
                        std::to_string(i) + " of level " + std::to_string(l) + " both use row " + std::to_string(x) +
                        ", one writing it";
        };
        std::vector<uint32_t> rd;
        for (size_t i = 0; i < ops_v.size(); ++i) {
            const uint32_t l = lv[i] / TAMD_COST_CLASSES;
            for (uint32_t k = ops_v[i].first; k < ops_v[i].first + ops_v[i].count; ++k) {
                const uint32_t kind = in[k].w0 & 0xff;
                if (kind == TAMD_I_STORE || kind == TAMD_I_STOREC) {
                    const uint64_t key = (uint64_t)l << 32 | in[k].row;
                    const auto it = writer.find(key);
                    if (it != writer.end() && it->second != i) bad(i, l, in[k].row, it->second);
                    writer[key] = (uint32_t)i;
                }
            }
        }
        for (size_t i = 0; i < ops_v.size(); ++i) {
            const uint32_t l = lv[i] / TAMD_COST_CLASSES;
            rd.clear();
            for (uint32_t k = ops_v[i].first; k < ops_v[i].first + ops_v[i].count; ++k) {
                const uint32_t kind = in[k].w0 & 0xff;
                if (kind == TAMD_I_ACC || kind == TAMD_I_ACC3) rd.push_back(in[k].row);
                else if (kind == TAMD_I_ACCR)
                    for (uint32_t q = 0; q < in[k].cap; ++q) rd.push_back(in[k].row + q * in[k + 1].row);
            }
            for (uint32_t x : rd) {
                const auto it = writer.find((uint64_t)l << 32 | x);
                if (it != writer.end() && it->second != i) bad(i, l, x, it->second);
            }
        }
    }

    void flush() {
        ctx.prepare_flush();
        check_levels();
        if (g_pipeline) check_pipeline();
        const auto& ops_v = ctx.pb.ops();
        const auto& lv = ctx.pb.op_levels();
        const uint32_t maxl = ctx.pb.max_level();
        std::vector<uint32_t> sorted;
        sorted.reserve(ops_v.size() * 4);
        // op_levels() holds buckets TAMD_COST_CLASSES * level + class; run level by level
        for (uint32_t l = 1; l <= maxl; ++l)
            for (size_t i = 0; i < ops_v.size(); ++i)
                if (lv[i] / TAMD_COST_CLASSES == l) {
                    const tamd_op& o = ops_v[i];
                    sorted.push_back(o.first); sorted.push_back(o.count);
                    sorted.push_back(o.span); sorted.push_back(o.full);
                }
        static const bool dump = getenv("CP_DUMP_OPS") != nullptr;
        if (dump && !ops_v.empty()) {  // (diagnostics) every op: level, instructions, rows read, stores
            const auto& in = ctx.pb.instrs();
            fprintf(stderr, "program %llu: %zu ops, %u levels\n", (unsigned long long)programs, ops_v.size(), maxl);
            for (size_t i = 0; i < ops_v.size(); ++i) {
                const tamd_op& o = ops_v[i];
                uint32_t rows = 0, runs = 0, acc3 = 0, stores = 0;
                for (uint32_t k = o.first; k < o.first + o.count; ++k) {
                    const uint32_t kind = in[k].w0 & 0xff;
                    if (kind == TAMD_I_ACC) ++rows;
                    else if (kind == TAMD_I_ACC3) { ++rows; ++acc3; }
                    else if (kind == TAMD_I_ACCR) { rows += in[k].cap; ++runs; }
                    else if (kind == TAMD_I_STORE || kind == TAMD_I_STOREC) ++stores;
                }
                fprintf(stderr, "  op L%u c%u: %u instrs, %u rows (%u acc3, %u runs), %u stores, span %u\n",
                        lv[i] / TAMD_COST_CLASSES, lv[i] % TAMD_COST_CLASSES, o.count, rows, acc3, runs, stores, o.span);
            }
        }
        static const bool rstats = getenv("CP_READ_STATS") != nullptr;
        if (rstats && !ops_v.empty()) {  // (diagnostics) rows read per run mode, and how many distinct
            const auto& in = ctx.pb.instrs();
            std::unordered_map<uint32_t, uint32_t> seen_dense, seen_all;
            uint64_t reads[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dense_ops = 0, dense_multi = 0;
            std::vector<uint32_t> op_rows;
            for (size_t i = 0; i < ops_v.size(); ++i) {
                const tamd_op& o = ops_v[i];
                bool has_dense = false;
                for (uint32_t k = o.first; k < o.first + o.count; ++k) {
                    const uint32_t kind = in[k].w0 & 0xff;
                    if (kind == TAMD_I_ACC || kind == TAMD_I_ACC3) {
                        reads[0]++;
                        seen_all[in[k].row]++;
                    } else if (kind == TAMD_I_ACCR) {
                        const uint32_t mode = (in[k].w0 >> 8) & 0xff, stride = in[k + 1].row;
                        for (uint32_t j = 0; j < in[k].cap; ++j) {
                            reads[mode]++;
                            seen_all[in[k].row + j * stride]++;
                            if (mode == TAMD_R_DENSE) seen_dense[in[k].row + j * stride]++;
                        }
                        if (mode == TAMD_R_DENSE) has_dense = true;
                    }
                }
                dense_ops += has_dense;
            }
            (void)dense_multi;
            g_rs[0] += reads[0]; g_rs[1] += reads[TAMD_R_LANE3]; g_rs[2] += reads[TAMD_R_CAUCHY];
            g_rs[3] += reads[TAMD_R_CONST]; g_rs[4] += reads[TAMD_R_MULTI]; g_rs[5] += reads[TAMD_R_DENSE];
            g_rs[6] += seen_dense.size(); g_rs[7] += seen_all.size(); g_rs[8] += dense_ops;
        }
        if (!ops_v.empty()) {
            const int rc = oracle_run_program(arena.data(), arena.size(), sorted.data(),
                                              (unsigned)(sorted.size() / 4),
                                              (const uint32_t*)ctx.pb.instrs().data(),
                                              (unsigned)ctx.pb.instrs().size());
            if (rc != 0 && error.empty()) error = "oracle_run_program failed rc=" + std::to_string(rc);
            ++programs;
            ops += ops_v.size();
            instrs += ctx.pb.instrs().size();
            levels += maxl;
        }
        resolve();
        const uint64_t done = ctx.epoch;
        ctx.finish_flush();
        // pipelined, a program completes only with later programs' launches: rows it freed are
        // reusable once its last level has run (the session releases by device completion events)
        ctx.rows.release_up_to(g_pipeline ? release_bound(done) : done);
    }

    void resolve() {
        char buf[256];
        for (const PendEnc& e : pend_enc) {
            const uint8_t* d = at(e.row);
            snprintf(buf, sizeof(buf), "E 0 %u %u %u %u %u %016llx", e.total, e.meta.Row, e.meta.ColumnStart,
                     e.meta.SumCount, e.meta.LDPCCount, (unsigned long long)fnv1a(d, e.total));
            lines[e.pos] = buf;
        }
        pend_enc.clear();
        for (size_t k = 0; k < pend_dec.size(); ++k) {
            std::string& ln = lines[pend_dec_pos[k]];
            for (const PendDec& dd : pend_dec[k]) {
                const uint8_t* d = at(dd.row);
                unsigned len = 0;
                const int hb = get_length_header(d, dd.upper, len);
                uint32_t packet = 0;
                if (hb < 1 || len + hb > dd.upper) { if (error.empty()) error = "bad recovered header"; continue; }
                (void)packet;
                snprintf(buf, sizeof(buf), ":%u:%016llx", len, (unsigned long long)fnv1a(d + hb, len));
                // placeholder "#" marks where the length/hash go
                const size_t at_pos = ln.find('#');
                if (at_pos != std::string::npos) ln.replace(at_pos, 1, buf);
            }
        }
        pend_dec.clear();
        pend_dec_pos.clear();
    }

    // ---- backend interface for run_stream ----
    struct RecRef { RecoveryOut out; };
    struct DecRef { };

    int enc_add(uint32_t index, uint32_t len, uint32_t* col) {
        cancel_ahead();
        uint32_t framed = 0, header = 0;
        const RowId r = write_original(index, len, &framed, &header);
        if (r == kNoRow) { error = "arena full"; return 5; }
        const Result rc = E()->add(r, framed, header, len, nullptr, col, g_contig);
        if (rc != kSuccess && !g_contig) ctx.rows.free_deferred(r);
        if (batch && (index + 1) % batch == 0) flush();
        return rc;
    }
    // batched adds (the session's path), off with nobatch=1
    bool enc_add_run(uint32_t index, uint32_t k, uint32_t len, uint32_t* col0) {
        if (g_nobatch) return false;
        cancel_ahead();
        std::vector<RowId> rows(k);
        uint32_t framed = 0, header = 0;
        for (uint32_t j = 0; j < k; ++j) {
            rows[j] = write_original(index + j, len, &framed, &header);
            if (rows[j] == kNoRow) { error = "arena full"; return false; }
        }
        if (!E()->add_run(rows.data(), k, framed, header, len, g_contig, col0)) {
            if (!g_contig)
                for (RowId r : rows) ctx.rows.free_deferred(r);
            return false;
        }
        if (batch && (index + k) / batch != index / batch) flush();
        return true;
    }
    bool dec_add_run(uint32_t col0, uint32_t index, uint32_t k, uint32_t len) {
        if (g_nobatch) return false;
        std::vector<RowId> rows(k);
        uint32_t framed = 0, header = 0;
        for (uint32_t j = 0; j < k; ++j) {
            rows[j] = write_original(index + j, len, &framed, &header, 1);
            if (rows[j] == kNoRow) { error = "arena full"; return false; }
        }
        if (!D()->add_run_inorder(col0, rows.data(), k, framed, header, len, g_contig)) {
            if (!g_contig)
                for (RowId r : rows) ctx.rows.free_deferred(r);
            return false;
        }
        return true;
    }
    // CP_TIME=1 (diagnostics): host nanoseconds in encode / add_recovery / is_ready / decode
    uint64_t t_ns[4] = {0, 0, 0, 0}, t_n[4] = {0, 0, 0, 0};
    static uint64_t tnow() {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    struct TScope {
        Harness& h;
        int k;
        uint64_t t0;
        TScope(Harness& hh, int kk) : h(hh), k(kk), t0(tnow()) {}
        ~TScope() { h.t_ns[k] += tnow() - t0; h.t_n[k]++; }
    };
    std::vector<RecoveryOut> spec;
    std::vector<Encoder::Mark> marks;  // marks[i]: the encoder before spec[i] was encoded
    size_t spec_next = 0;
    uint32_t depth = 1;
    bool last_enc = false;
    uint64_t ahead_used = 0, ahead_rewound = 0;
    void cancel_ahead() {
        if (spec_next < spec.size()) {
            E()->rewind(marks[spec_next]);
            for (size_t i = spec_next; i < spec.size(); ++i) ctx.rows.free_deferred(spec[i].row);
            ahead_rewound += spec.size() - spec_next;
            depth = 1;
        }
        spec.clear();
        marks.clear();
        spec_next = 0;
        last_enc = false;
    }
    int enc_encode(RecRef& r) {
        TScope ts(*this, 0);
        if (g_ahead) {
            if (spec_next < spec.size()) {
                r.out = spec[spec_next++];
                ++ahead_used;
                return 0;
            }
            if (!spec.empty()) {
                depth = depth * 2 < g_ahead ? depth * 2 : g_ahead;
                spec.clear();
                marks.clear();
                spec_next = 0;
            }
        }
        const int rc = E()->encode(r.out);
        if (g_ahead && rc == kSuccess && last_enc) {
            for (uint32_t k = 0; k < depth && E()->encode_is_quiet(); ++k) {
                const Encoder::Mark m = E()->mark();
                RecoveryOut o;
                if (E()->encode(o) != kSuccess) {
                    E()->rewind(m);
                    break;
                }
                marks.push_back(m);
                spec.push_back(o);
            }
        }
        last_enc = rc == kSuccess;
        return rc;
    }
    int enc_ack(const uint8_t* buf, uint32_t n, uint32_t* next) {
        cancel_ahead();
        return E()->acknowledge(buf, n, next);
    }
    int enc_is_ready() { return E()->remaining_slots() <= 2 ? (int)kMaxPacketsReached : 0; }
    int dec_add_original(uint32_t col, uint32_t index, uint32_t len) {
        uint32_t framed = 0, header = 0;
        const RowId r = write_original(index, len, &framed, &header, 1);
        if (r == kNoRow) { error = "arena full"; return 5; }
        bool took = false;
        const Result rc = D()->add_original(col, r, framed, header, len, nullptr, &took, g_contig);
        if (!took && !g_contig) ctx.rows.free_deferred(r);
        return rc;
    }
    void recovery_lost(const RecRef& r) { ctx.rows.free_deferred(r.out.row); }

    int dec_add_recovery(const RecRef& r) {
        bool took = false;
        // Footer parsing reads only the footer bytes at the end of the packet, which the
        // encoder produced on the host; the data bytes in front of it are not needed.
        uint8_t tail[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint32_t tl = r.out.total() < 8 ? r.out.total() : 8;
        memcpy(tail + tl - r.out.footer_len, r.out.footer, r.out.footer_len);
        TScope ts(*this, 1);
        const Result rc = D()->add_recovery(r.out.row, r.out.total(), tail, nullptr, &took);
        if (!took) ctx.rows.free_deferred(r.out.row);
        return rc;
    }
    int dec_is_ready() {
        TScope ts(*this, 2);
        return D()->is_ready();
    }
    int dec_decode(std::vector<uint32_t>& nums, DecRef&) {
        std::vector<RecoveredPacket*> got;
        Result rc;
        {
            TScope ts(*this, 3);
            rc = D()->decode(got);
        }
        if (rc == kSuccess) {
            pend_dec.emplace_back();
            for (RecoveredPacket* rp : got) {
                nums.push_back(rp->packet_num);
                pend_dec.back().push_back(PendDec{rp->row, rp->framed_upper, 0});
            }
        }
        return rc;
    }
    int dec_ack(uint8_t* buf, uint32_t limit, uint32_t* used) { return D()->ack(buf, limit, used); }
    void stats(uint64_t e[9], uint64_t d[11]) {
        cancel_ahead();
        E()->stats(e, 9);
        D()->stats(d, 11);
    }
    uint64_t vclock = 0;
    void set_time(uint64_t ms) {
        if (!vclock) enc->set_clock(&vclock);
        vclock = ms;
    }
    int enc_retransmit(uint32_t* num, uint32_t* bytes, const uint8_t** data) {
        cancel_ahead();
        StoredOriginal ov;
        const StoredOriginal* o = &ov;
        const Result rc = E()->retransmit(&ov);
        if (rc == kSuccess) {
            *num = o->column;
            *bytes = o->bytes - o->header_bytes;
            *data = nullptr;
        }
        return rc;
    }

    // ---- transcript interface ----
    void on_encode(int rc, const RecRef& r) {
        if (rc != 0) { lines.push_back("E " + std::to_string(rc)); return; }
        pend_enc.push_back(PendEnc{r.out.row, r.out.total(), r.out.meta, lines.size()});
        lines.push_back("E ?");
        if (sync) flush();
    }
    void on_decode(int rc, const std::vector<uint32_t>& nums, const DecRef&) {
        std::string ln = "D " + std::to_string(rc) + " " + std::to_string(nums.size());
        for (uint32_t n : nums) ln += " " + std::to_string(n) + "#";
        if (rc == 0) pend_dec_pos.push_back(lines.size());
        lines.push_back(ln);
        if (sync) flush();
    }
    void on_ack(int rd, const uint8_t* buf, uint32_t used, int re, uint32_t next) {
        char b[128];
        snprintf(b, sizeof(b), "K %d %u %016llx %d %u", rd, used, (unsigned long long)fnv1a(buf, used), re, next);
        lines.push_back(b);
    }
    void on_event(char kind, int rc, uint32_t a, uint32_t b) {
        if (rc == 0) return;
        char t[64];
        snprintf(t, sizeof(t), "%c %d %u %u", kind, rc, a, b);
        lines.push_back(t);
    }
    void on_retransmit(int rc, uint32_t num, uint32_t bytes, uint64_t h) {
        TextSink t;
        fmt_retransmit(t, rc, num, bytes, h);
        t.text.pop_back();
        lines.push_back(t.text);
    }
    void on_stats(const uint64_t e[9], const uint64_t d[11]) {
        flush();
        TextSink t;
        fmt_stats(t, e, d);
        std::string s = t.text;
        if (!s.empty() && s.back() == '\n') s.pop_back();
        lines.push_back(s);
    }
};

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: cp_harness <out> k=v...\n"); return 2; }
    if (!gf_init()) { fprintf(stderr, "gf_init failed\n"); return 3; }
    if (oracle_self_test() != 0) { fprintf(stderr, "oracle self test failed\n"); return 3; }
    Params p;
    bool sync = true;
    uint32_t batch = 0;
    for (int i = 2; i < argc; ++i) {
        const char* eq = strchr(argv[i], '=');
        if (!eq) return 2;
        std::string k(argv[i], eq - argv[i]);
        const char* vs = eq + 1;
        const unsigned long long v = strtoull(vs, nullptr, 0);
        if (k == "mode") sync = strcmp(vs, "sync") == 0;
        else if (k == "batch") batch = (uint32_t)v;
        else if (k == "arena_mb") g_arena_bytes = v << 20;
        else if (k == "dirty") g_dirty = v != 0;
        else if (k == "nobatch") g_nobatch = v != 0;
        else if (k == "pipeline") g_pipeline = v != 0;
        else if (k == "drain") g_drain = (uint32_t)v;
        else if (k == "expand") g_expand = (uint32_t)v;
        else if (k == "backsub") g_backsub = (uint32_t)v;
        else if (k == "split") g_split = (uint32_t)v;
        else if (k == "contig") g_contig = v != 0;
        else if (k == "ahead") g_ahead = (uint32_t)v;
        else if (k == "short") g_short = v != 0;
        else if (k == "ddirect") g_ddirect = (int)v;
        else if (parse_param(p, k, v)) {}
        else { fprintf(stderr, "bad key %s\n", k.c_str()); return 2; }
    }
    Harness h(p);
    h.sync = sync;
    h.batch = sync ? 0 : (batch ? batch : 1u << 30);
    Summary s = run_stream(p, h, h);
    h.flush();
    FILE* f = fopen(argv[1], "wb");
    if (!f) return 4;
    for (const std::string& l : h.lines) fprintf(f, "%s\n", l.c_str());
    fprintf(f, "Z originals=%llu lost=%llu recoveries=%llu lostrec=%llu recovered=%llu arq=%llu "
               "acks=%llu decodes=%llu flush=%llu missing=%llu bad=0\n",
            (unsigned long long)s.originals, (unsigned long long)s.lost_originals,
            (unsigned long long)s.recoveries, (unsigned long long)s.lost_recoveries,
            (unsigned long long)s.recovered, (unsigned long long)s.arq_redelivered,
            (unsigned long long)s.acks, (unsigned long long)s.decode_calls,
            (unsigned long long)s.flush_encodes, (unsigned long long)s.missing_at_end);
    fclose(f);
    if (getenv("CP_TIME"))
        fprintf(stderr, "host us: encode %.1f ms / %llu, add_recovery %.1f ms / %llu, is_ready %.1f ms / %llu, decode %.1f ms / %llu\n",
                h.t_ns[0] * 1e-6, (unsigned long long)h.t_n[0], h.t_ns[1] * 1e-6, (unsigned long long)h.t_n[1],
                h.t_ns[2] * 1e-6, (unsigned long long)h.t_n[2], h.t_ns[3] * 1e-6, (unsigned long long)h.t_n[3]);
    fprintf(stderr, "programs=%llu ops=%llu instrs=%llu levels=%llu live_rows=%zu pipelined_pairs=%llu\n",
            (unsigned long long)h.programs, (unsigned long long)h.ops, (unsigned long long)h.instrs,
            (unsigned long long)h.levels, h.ctx.rows.live_rows(), (unsigned long long)h.pipelined_pairs);
#ifdef TAMD_PROF
    for (int i = 0; i < prof::kSlots; ++i)
        if (prof::calls[i])
            fprintf(stderr, "%-14s calls %10llu  Mcyc %10.2f  cyc/call %10.0f\n", prof::names[i],
                    (unsigned long long)prof::calls[i], prof::cycles[i] / 1e6, (double)prof::cycles[i] / prof::calls[i]);
#endif
    if (g_ahead)
        fprintf(stderr, "ahead: used=%llu rewound=%llu\n", (unsigned long long)h.ahead_used,
                (unsigned long long)h.ahead_rewound);
    if (getenv("CP_READ_STATS"))
        fprintf(stderr, "reads: acc %llu lane3 %llu cauchy %llu const %llu multi %llu dense %llu; distinct dense %llu, "
                "distinct all %llu; ops with dense runs %llu\n",
                (unsigned long long)g_rs[0], (unsigned long long)g_rs[1], (unsigned long long)g_rs[2],
                (unsigned long long)g_rs[3], (unsigned long long)g_rs[4], (unsigned long long)g_rs[5],
                (unsigned long long)g_rs[6], (unsigned long long)g_rs[7], (unsigned long long)g_rs[8]);
    if (!h.error.empty()) { fprintf(stderr, "error: %s\n", h.error.c_str()); return 6; }
    return 0;
}
