// workload.h -- the synthetic Siamese FEC workload.
//
// One "stream" is one connection: an encoder and a decoder joined by a lossy channel.  The
// driver feeds originals, emits recovery packets at rate f with a token bucket (Tonk's rule,
// TonkineseBandwidth.cpp:248-293), drops packets with a seeded loss process, exchanges
// acknowledgements every A originals, re-delivers originals still missing after an ARQ lag,
// and finally flushes recovery packets until every original is received or recovered.
//
// The driver is a template over a codec backend so that the SAME event sequence runs against
//   * the reference codec (oracle/_ref, golden fixtures and the CPU baseline),
//   * the MI355X engine through the siamese.h C-ABI, and
//   * the MI355X engine's batched device-resident session (bench).
// All decisions use integer arithmetic so every compiler produces the same sequence.
#pragma once

#include <stdint.h>
#include <string.h>
#include <vector>
#include <string>
#include <algorithm>

namespace tamd {
namespace wl {

// PCG32 (same generator the codec uses for LDPC columns, SiameseTools.h:79-101).
struct Pcg {
    uint64_t state = 0, inc = 0;
    void seed(uint64_t y, uint64_t x) {
        state = 0;
        inc = (y << 1u) | 1u;
        next();
        state += x;
        next();
    }
    uint32_t next() {
        const uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
        const uint32_t rot = (uint32_t)(old >> 59);
        return (xs >> rot) | (xs << ((uint32_t)(-(int32_t)rot) & 31u));
    }
};

struct Params {
    uint32_t stream_id = 0;
    uint32_t n_originals = 256;
    uint32_t payload_min = 1300, payload_max = 1300;
    // Loss process over send events (originals and, if enabled, recovery packets).
    // Uniform: lost iff draw < loss_thresh.  Gilbert-Elliott (ge_enable): the state flips
    // good->bad with probability gb_thresh/2^32 and bad->good with bg_thresh/2^32 before
    // each event; a packet is lost iff the state is bad.
    uint32_t loss_thresh = 0;
    uint32_t ge_enable = 0, gb_thresh = 0, bg_thresh = 0;
    uint32_t loss_on_recovery = 1;
    // Recovery rate in 1/65536 units per original (Tonk: f = max(2p, 1%)).
    uint32_t fec_rate_q16 = 655;
    uint32_t ack_every = 0;    // 0: no acknowledgements
    uint32_t ack_bytes = 256;  // decoder ack buffer size (>= SIAMESE_ACK_MIN_BYTES)
    uint32_t arq_lag = 0;      // 0: no ARQ
    uint32_t flush_max = 4096; // cap on end-of-stream recovery packets
    // Retransmission (siamese_encoder_retransmit, SiameseEncoder.cpp:877-1044) under a virtual
    // millisecond clock: every rtx_every originals the sender asks for up to kRtxPerTick
    // retransmissions and sends them through the lossy channel; the clock advances rtx_msec per
    // original so RTO decisions are deterministic.  0: off (the codec's own clock is used).
    uint32_t rtx_every = 0, rtx_msec = 1;
    uint32_t batch_adds = 1;   // runs of quiet originals go to the backend as batched adds
    // Window-full behaviour (siamese.cpp:80-93, SiameseEncoder.cpp:91-96): before every add the
    // sender asks siamese_encoder_is_ready and logs a refusal ("W" line) but adds anyway (the
    // two slots of slack); an add refused with MaxPacketsReached makes the receiver acknowledge
    // (and, if that frees nothing, the sender flush a recovery packet) before the add is retried.
    // Single adds only (the window's fill is the codec's, not the runner's, to know).
    uint32_t hold_full = 0;
    uint64_t seed_data = 1000, seed_loss = 2000;
};

// Packet numbers are 22-bit columns (SiameseCommon.h:102 kColumnPeriod): the stream index of
// column `col` when `top` originals have been added, the most recent one at or below top - 1
// (recovered and retransmitted originals are always in the encoder's window, < 2^21 back).
inline uint32_t index_of_column(uint32_t col, uint32_t top) {
    const uint32_t last = top ? top - 1 : 0;
    return last - ((last - col) & 0x3fffffu);
}

static const uint32_t kRtxPerTick = 4;
static const uint64_t kVirtualClockStart = 1000;  // ms (send times are never 0)

// key=value workload arguments shared by every driver (golden_gen, cp_harness, cp_bench).
// Returns false for an unknown key.
inline bool parse_param(Params& p, const std::string& k, unsigned long long v) {
    if (k == "stream") p.stream_id = (uint32_t)v;
    else if (k == "n") p.n_originals = (uint32_t)v;
    else if (k == "pmin") p.payload_min = (uint32_t)v;
    else if (k == "pmax") p.payload_max = (uint32_t)v;
    else if (k == "loss") p.loss_thresh = (uint32_t)v;
    else if (k == "ge") p.ge_enable = (uint32_t)v;
    else if (k == "gb") p.gb_thresh = (uint32_t)v;
    else if (k == "bg") p.bg_thresh = (uint32_t)v;
    else if (k == "lossrec") p.loss_on_recovery = (uint32_t)v;
    else if (k == "fec") p.fec_rate_q16 = (uint32_t)v;
    else if (k == "ack") p.ack_every = (uint32_t)v;
    else if (k == "ackbytes") p.ack_bytes = (uint32_t)v;
    else if (k == "arq") p.arq_lag = (uint32_t)v;
    else if (k == "flush") p.flush_max = (uint32_t)v;
    else if (k == "rtx") p.rtx_every = (uint32_t)v;
    else if (k == "rtxms") p.rtx_msec = (uint32_t)v;
    else if (k == "full") p.hold_full = (uint32_t)v;
    else if (k == "seed_data") p.seed_data = v;
    else if (k == "seed_loss") p.seed_loss = v;
    else return false;
    return true;
}

// Payload bytes of original i (index within the stream).  Length and contents come from a
// PCG stream seeded with (seed_data, i) so any packet can be regenerated independently (the
// device generator in the bench uses the same definition, kernels.hip tamd_gen_rows).
inline uint32_t payload_length(const Params& p, uint32_t i) {
    if (p.payload_min == p.payload_max) return p.payload_min;
    Pcg g;
    g.seed(p.seed_data ^ 0x5bd1e995u, i);
    return p.payload_min + g.next() % (p.payload_max - p.payload_min + 1);
}

inline void payload_bytes(const Params& p, uint32_t i, uint8_t* out, uint32_t len) {
    Pcg g;
    g.seed(p.seed_data, i);
    uint32_t k = 0;
    for (; k + 4 <= len; k += 4) {
        const uint32_t w = g.next();
        memcpy(out + k, &w, 4);
    }
    if (k < len) {
        const uint32_t w = g.next();
        memcpy(out + k, &w, len - k);
    }
}

// FNV-1a 64-bit, used for transcript digests.
inline uint64_t fnv1a(const uint8_t* d, size_t n, uint64_t h = 1469598103934665603ULL) {
    for (size_t i = 0; i < n; ++i) { h ^= d[i]; h *= 1099511628211ULL; }
    return h;
}

// The loss process is a fixed sequence of draws (one per packet sent through the channel, in
// send order).  The draws are generated ahead, as a bitmap (bit i: draw i is a loss), so that
// scenario generation stays outside a timed region ("timer around the API calls
// only") and a run of delivered originals is found a 64-bit word at a time.  Draws past the
// generated ones are produced on demand, continuing the same PCG sequence: the channel's answers
// never depend on how far ahead it was generated.
struct LossChannel {
    Pcg rng;
    bool bad = false;
    const Params* p = nullptr;
    std::vector<uint64_t> bits;
    uint64_t pos = 0, avail = 0;  // next draw; draws generated
    void init(const Params& prm) {
        p = &prm;
        rng.seed(prm.seed_loss, 0);
        bad = false;
        bits.clear();
        pos = avail = 0;
    }
    // Generate draws up to `n` (at least).
    void generate(uint64_t n) {
        n = (n + 63) & ~63ull;
        if (n <= avail) return;
        bits.resize(n / 64, 0);
        for (uint64_t i = avail; i < n; i += 64) {
            uint64_t w = 0;
            for (unsigned b = 0; b < 64; ++b) w |= (uint64_t)draw() << b;
            bits[i / 64] = w;
        }
        avail = n;
    }
    bool lost() {
        if (pos >= avail) generate(avail + 4096);
        const bool l = (bits[pos >> 6] >> (pos & 63)) & 1u;
        ++pos;
        return l;
    }
    // Consume the next draws up to and including the first loss among the next `kmax`: returns
    // its index (< kmax), or kmax when all kmax are deliveries (kmax draws consumed).
    uint32_t first_lost(uint32_t kmax) {
        if (pos + kmax > avail) generate(pos + kmax + 4096);
        uint64_t at = pos;
        const uint64_t end = pos + kmax;
        while (at < end) {
            const uint64_t w = bits[at >> 6] >> (at & 63);
            if (w) {
                const uint64_t hit = at + (uint64_t)__builtin_ctzll(w);
                if (hit < end) {
                    pos = hit + 1;
                    return (uint32_t)(hit - (end - kmax));
                }
                break;
            }
            at = (at | 63) + 1;
        }
        pos = end;
        return kmax;
    }

private:
    bool draw() {
        const uint32_t u = rng.next();
        if (!p->ge_enable) return u < p->loss_thresh;
        if (bad) { if (u < p->bg_thresh) bad = false; }
        else     { if (u < p->gb_thresh) bad = true; }
        return bad;
    }
};

// Counters every backend reports identically.
struct Summary {
    uint64_t originals = 0, lost_originals = 0, recoveries = 0, lost_recoveries = 0;
    uint64_t recovered = 0, arq_redelivered = 0, acks = 0, decode_calls = 0, flush_encodes = 0;
    uint64_t retransmits = 0;
    uint64_t missing_at_end = 0;
};

// Backend concept (all methods return siamese.h result codes, 0 = success):
//   typedef RecRef, DecRef
//   int  enc_add(uint32_t index, uint32_t len, uint32_t* packetNumOut)
//   int  enc_encode(RecRef& out)              -- out describes the recovery packet
//   int  enc_ack(const uint8_t* buf, uint32_t n, uint32_t* nextExpected)
//   int  dec_add_original(uint32_t packetNum, uint32_t index, uint32_t len)
//   int  dec_add_recovery(const RecRef& r)
//   void recovery_lost(const RecRef& r)       -- the channel dropped the packet
//   int  dec_is_ready()
//   int  dec_decode(std::vector<uint32_t>& packetNums, DecRef& out)
//   int  dec_ack(uint8_t* buf, uint32_t limit, uint32_t* used)
//   void stats(uint64_t enc[9], uint64_t dec[11])
//   void set_time(uint64_t msec)               -- virtual clock (retransmit scenarios only)
//   int  enc_is_ready()                        -- siamese_encoder_is_ready (hold_full only)
//   int  enc_retransmit(uint32_t* packetNum, uint32_t* bytes, const uint8_t** data)
//                                              -- data may be null (the runner regenerates it)
//   bool enc_add_run(uint32_t index, uint32_t k, uint32_t len, uint32_t* firstPacketNum)
//   bool dec_add_run(uint32_t packetNum, uint32_t index, uint32_t k, uint32_t len)
//        batched adds of k consecutive originals (all delivered, no event among them): each
//        returns false, with nothing done, when it cannot give exactly the result of k single
//        calls (for dec_add_run: k add_original calls each followed by an is_ready that reports
//        NeedMoreData); the runner then makes the single calls.  A backend without batching
//        returns false.
// Transcript concept:
//   on_encode(int rc, const RecRef&), on_decode(int rc, nums, const DecRef&), on_ack(...),
//   on_event(char kind, int rc, uint32_t a, uint32_t b), on_stats(enc, dec),
//   on_retransmit(int rc, uint32_t packetNum, uint32_t bytes, uint64_t payload digest)
template <class Backend, class Transcript>
class Runner {
public:
    Runner(const Params& p, Backend& be, Transcript& tr) : p_(p), be_(be), tr_(tr) {
        ch_.init(p_);
        ack_countdown_ = p_.ack_every;
        rtx_countdown_ = p_.rtx_every;
        now_ms_ = kVirtualClockStart;
        have_.assign(p_.n_originals, 0);
        col_of_.assign(p_.n_originals, 0);
    }

    uint32_t position() const { return next_; }
    const Summary& summary() const { return s_; }
    // Scenario generation, done before any timed region: the loss draws of the originals and of
    // the recovery packets sent with them (the channel continues the sequence on demand past it).
    void pregenerate() {
        const uint64_t rec = (uint64_t)p_.n_originals * p_.fec_rate_q16 / 65536u;
        ch_.generate((uint64_t)p_.n_originals + 2 * rec + 1024);
    }

    // Feed the next `n` originals (and everything they trigger).  Runs of originals that trigger
    // nothing (delivered, no recovery packet, acknowledgement, retransmission or ARQ due after
    // them) go to the backend as batched adds; the calls and results are those of single adds.
    void advance(uint32_t n) {
        const uint32_t end = std::min(p_.n_originals, next_ + n);
        const bool batching = p_.batch_adds && !p_.rtx_every && !p_.hold_full && p_.payload_min == p_.payload_max;
        while (next_ < end) {
            int drawn = -1;  // loss draw of original next_ made by quiet_run (-1: not drawn)
            if (batching) {
                const uint32_t k = quiet_run(end, drawn);
                if (k >= 1 && next_ + k < end) {
                    // the quiet run and the original after it (lost, or the one an event follows)
                    // as one batch of adds, then that original's events
                    if (drawn < 0) drawn = ch_.lost() ? 1 : 0;  // (its draw, as one() makes it)
                    run_with_event(next_, k, drawn != 0);
                    next_ += k + 1;
                    continue;
                }
                if (k > 1) {
                    run_quiet(next_, k);
                    next_ += k;
                } else if (k == 1) {
                    one(next_++, 0);
                }
                if (next_ >= end) break;
            }
            one(next_++, drawn);
        }
    }

    // End of stream: lossless recovery packets until the decoder has everything, then stats.
    void finish() {
        advance(p_.n_originals);
        for (uint32_t k = 0; k < p_.flush_max; ++k) {
            // (have_ only ever gains entries: the first missing index only moves up)
            while (scan_ < p_.n_originals && have_[scan_]) ++scan_;
            if (scan_ == p_.n_originals) break;
            ++s_.flush_encodes;
            send_recovery(false);
        }
        for (uint32_t i = 0; i < p_.n_originals; ++i) if (!have_[i]) ++s_.missing_at_end;
        uint64_t es[9] = {0}, ds[11] = {0};
        be_.stats(es, ds);
        tr_.on_stats(es, ds);
    }

private:
    const Params& p_;
    Backend& be_;
    Transcript& tr_;
    Summary s_;
    LossChannel ch_;
    std::vector<uint8_t> have_;
    std::vector<uint32_t> col_of_, pending_arq_;
    size_t arq_head_ = 0;
    uint32_t tokens_ = 0, next_ = 0;
    uint32_t top_ = 0;   // originals added to the encoder (index_of_column)
    uint32_t scan_ = 0;  // finish(): every index below is delivered or recovered
    uint32_t ack_countdown_ = 0;  // originals until the next acknowledgement
    uint32_t rtx_countdown_ = 0;  // originals until the next retransmission tick
    uint64_t now_ms_ = 0;         // virtual clock (rtx_every > 0)
    std::vector<uint32_t> nums_;
    std::vector<uint8_t> rtx_buf_;

    // Retransmission tick (Tonk's PostRetransmit, TonkineseOutgoing.cpp:1079-1100): up to
    // kRtxPerTick originals chosen by the encoder's RTO logic, each sent through the channel.
    // Packet numbers are stream indices modulo the 22-bit column period.
    void retransmit_tick() {
        for (uint32_t k = 0; k < kRtxPerTick; ++k) {
            uint32_t num = 0, bytes = 0;
            const uint8_t* data = nullptr;
            const int rc = be_.enc_retransmit(&num, &bytes, &data);
            uint64_t h = 0;
            const uint32_t idx = index_of_column(num, top_);
            if (rc == 0) {
                if (!data && idx < p_.n_originals) {
                    rtx_buf_.resize(bytes ? bytes : 1);
                    payload_bytes(p_, idx, rtx_buf_.data(), bytes);
                    data = rtx_buf_.data();
                }
                h = data ? fnv1a(data, bytes) : 0;
            }
            tr_.on_retransmit(rc, num, bytes, h);
            if (rc != 0) break;
            ++s_.retransmits;
            if (ch_.lost() || idx >= p_.n_originals) continue;
            const int ro = be_.dec_add_original(num, idx, bytes);
            tr_.on_event('T', ro, num, 0);
            if (!have_[idx]) have_[idx] = 1;
            decode_loop();
        }
    }

    void decode_loop() {
        while (be_.dec_is_ready() == 0) {
            nums_.clear();
            typename Backend::DecRef dref;
            const int rc = be_.dec_decode(nums_, dref);
            ++s_.decode_calls;
            tr_.on_decode(rc, nums_, dref);
            if (rc != 0) break;
            for (uint32_t c : nums_) {
                const uint32_t i = index_of_column(c, top_);
                if (i < p_.n_originals && !have_[i]) { have_[i] = 1; ++s_.recovered; }
            }
            if (nums_.empty()) break;
        }
    }

    void send_recovery(bool lossy) {
        typename Backend::RecRef r;
        const int rc = be_.enc_encode(r);
        tr_.on_encode(rc, r);
        if (rc != 0) return;
        ++s_.recoveries;
        if (lossy && p_.loss_on_recovery && ch_.lost()) {
            ++s_.lost_recoveries;
            be_.recovery_lost(r);
            return;
        }
        const int rr = be_.dec_add_recovery(r);
        tr_.on_event('R', rr, 0, 0);
        decode_loop();
    }

    // Length of the quiet run starting at next_ (at most end - next_): originals that are not
    // lost and after which no recovery packet, acknowledgement or ARQ redelivery is due.  The
    // channel is drawn for each of them; when the run ends at a lost original, that draw is
    // returned in `drawn_next` (1) for the original's own call.
    uint32_t quiet_run(uint32_t end, int& drawn_next) {
        uint32_t kmax = end - next_;
        if (p_.fec_rate_q16) {
            const uint32_t room = (65535u - tokens_) / p_.fec_rate_q16;  // tokens stay below 65536
            if (room < kmax) kmax = room;
        }
        if (p_.ack_every && ack_countdown_ - 1 < kmax) kmax = ack_countdown_ - 1;
        if (p_.arq_lag && arq_head_ < pending_arq_.size()) {
            const uint32_t due = pending_arq_[arq_head_] + p_.arq_lag;  // first index with ARQ
            const uint32_t room = due > next_ ? due - next_ : 0;
            if (room < kmax) kmax = room;
        }
        const uint32_t j = ch_.first_lost(kmax);
        if (j < kmax) drawn_next = 1;
        return j;
    }

    // k quiet originals from index i0 (every channel draw already made: all delivered).
    void run_quiet(uint32_t i0, uint32_t k) {
        const uint32_t len = payload_length(p_, i0);
        uint32_t col0 = 0;
        if (!be_.enc_add_run(i0, k, len, &col0)) {
            for (uint32_t j = 0; j < k; ++j) one(i0 + j, 0);
            return;
        }
        top_ = i0 + k;
        // (col_of_ is read only for lost originals, by ARQ: delivered runs do not store theirs)
        s_.originals += k;
        if (be_.dec_add_run(col0, i0, k, len)) {
            memset(&have_[i0], 1, k);
        } else {
            for (uint32_t j = 0; j < k; ++j) {
                const uint32_t col = (col0 + j) & 0x3fffffu;
                const int ro = be_.dec_add_original(col, i0 + j, len);
                tr_.on_event('O', ro, col, 0);
                have_[i0 + j] = 1;
                decode_loop();
            }
        }
        tokens_ += k * p_.fec_rate_q16;
        if (p_.ack_every) ack_countdown_ -= k;
    }

    // k quiet originals from i0 and original e = i0 + k after them (`lost`: its channel draw):
    // the encoder adds all k + 1 in one batch and the decoder the delivered ones; then e's
    // recovery tokens, acknowledgement and ARQ, exactly as one(e) does them.  The two codecs
    // only meet through recovery packets and acknowledgements, which come after e in both orders,
    // so adding e to the encoder before the run reaches the decoder changes no call's result.
    void run_with_event(uint32_t i0, uint32_t k, bool lost) {
        const uint32_t e = i0 + k;
        const uint32_t len = payload_length(p_, i0);
        uint32_t col0 = 0;
        if (!be_.enc_add_run(i0, k + 1, len, &col0)) {
            run_quiet(i0, k);
            one(e, lost ? 1 : 0);
            return;
        }
        top_ = e + 1;
        col_of_[e] = (col0 + k) & 0x3fffffu;  // (ARQ reads the lost ones' only)
        s_.originals += k + 1;
        const uint32_t kd = lost ? k : k + 1;  // delivered
        if (be_.dec_add_run(col0, i0, kd, len)) {
            memset(&have_[i0], 1, kd);
        } else {
            for (uint32_t j = 0; j < kd; ++j) {
                const uint32_t col = (col0 + j) & 0x3fffffu;
                const int ro = be_.dec_add_original(col, i0 + j, len);
                tr_.on_event('O', ro, col, 0);
                have_[i0 + j] = 1;
                decode_loop();
            }
        }
        if (lost) {
            ++s_.lost_originals;
            pending_arq_.push_back(e);
        }
        tokens_ += k * p_.fec_rate_q16;
        if (p_.ack_every) ack_countdown_ -= k;
        events_after(e);
    }

    // The decoder's acknowledgement, delivered to the encoder.
    void exchange_ack() {
        uint8_t buf[2048];
        const uint32_t limit = p_.ack_bytes < sizeof(buf) ? p_.ack_bytes : (uint32_t)sizeof(buf);
        uint32_t used = 0;
        const int rd = be_.dec_ack(buf, limit, &used);
        uint32_t next = 0;
        int re = -1;
        if (rd == 0 && used > 0) re = be_.enc_ack(buf, used, &next);
        tr_.on_ack(rd, buf, used, re, next);
        ++s_.acks;
    }

    // One original: add, channel, recovery tokens, acknowledgement, retransmission, ARQ.
    // `drawn`: its loss draw when already made (0 delivered, 1 lost), -1 to draw here.
    void one(uint32_t i, int drawn = -1) {
        if (p_.rtx_every) {
            now_ms_ += p_.rtx_msec;
            be_.set_time(now_ms_);
        }
        const uint32_t len = payload_length(p_, i);
        uint32_t col = 0;
        if (p_.hold_full) {
            const int ready = be_.enc_is_ready();
            tr_.on_event('W', ready, i, 0);
        }
        int ra = be_.enc_add(i, len, &col);
        tr_.on_event('a', ra, i, col);
        // window full (hold_full): the receiver acknowledges, and if that frees no slot the
        // sender flushes a recovery packet, until the add goes through (bounded)
        for (uint32_t tries = 0; p_.hold_full && ra == 3 && tries < 64; ++tries) {
            exchange_ack();
            ra = be_.enc_add(i, len, &col);
            tr_.on_event('a', ra, i, col);
            if (ra == 3) send_recovery(false);
        }
        if (ra == 0) top_ = i + 1;
        if (p_.hold_full && ra != 0) {  // never went out (the receiver does not expect it)
            have_[i] = 1;
            return;
        }
        col_of_[i] = col;
        ++s_.originals;
        if (drawn >= 0 ? drawn != 0 : ch_.lost()) {
            ++s_.lost_originals;
            pending_arq_.push_back(i);
        } else {
            const int ro = be_.dec_add_original(col, i, len);
            tr_.on_event('O', ro, col, 0);
            if (!have_[i]) have_[i] = 1;
            decode_loop();
        }

        events_after(i);
    }

    // What follows original i: recovery tokens, acknowledgement, retransmission tick, ARQ.
    void events_after(uint32_t i) {
        tokens_ += p_.fec_rate_q16;
        while (tokens_ >= 65536u) {
            tokens_ -= 65536u;
            send_recovery(true);
        }

        if (p_.ack_every && --ack_countdown_ == 0) {
            ack_countdown_ = p_.ack_every;
            exchange_ack();
        }

        if (p_.rtx_every && --rtx_countdown_ == 0) {
            rtx_countdown_ = p_.rtx_every;
            retransmit_tick();
        }

        if (p_.arq_lag) {
            while (arq_head_ < pending_arq_.size() && i - pending_arq_[arq_head_] >= p_.arq_lag) {
                const uint32_t j = pending_arq_[arq_head_++];
                if (!have_[j]) {
                    const int ro = be_.dec_add_original(col_of_[j], j, payload_length(p_, j));
                    tr_.on_event('X', ro, col_of_[j], 0);
                    have_[j] = 1;
                    ++s_.arq_redelivered;
                    decode_loop();
                }
            }
        }
    }
};

template <class Backend, class Transcript>
Summary run_stream(const Params& p, Backend& be, Transcript& tr) {
    Runner<Backend, Transcript> r(p, be, tr);
    r.finish();
    return r.summary();
}

} // namespace wl
} // namespace tamd
