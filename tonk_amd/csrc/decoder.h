// decoder.h -- Siamese decoder control plane (restates SiameseDecoder.h/.cpp of the reference).
//
// Window of received originals with per-subwindow got-bitmaps, sorted recovery-packet list,
// checked region, recovery-matrix generation, incremental Gaussian elimination with pivoting,
// running-sum elimination of received data, lower-triangle and back substitution, NACK ack
// generation and window removal -- all decisions identical to the reference.  The bulk row
// operations are symbolic (engine.h): after a successful solve each recovered original is one
// combine op over "partial" rows (received recovery rows with the known data eliminated).
#pragma once

#include "encoder.h"

#include <stdint.h>
#include <string.h>
#include <vector>

namespace tamd {

struct RecoveredPacket {
    uint32_t packet_num = 0;
    RowId row = kNoRow;          // framed row (varint len || payload) in the arena
    uint32_t framed_upper = 0;   // bytes the row may hold (exact once the length is read back)
    void* host = nullptr;        // C-ABI: host copy filled after readback
    uint32_t data_bytes = 0;     // payload length (valid after readback)
    uint32_t header_bytes = 0;
};

class Decoder : public FlushClient {
public:
    Decoder(Context* ctx, uint32_t row_bytes, HostRelease release = nullptr, void* user = nullptr);
    ~Decoder();

    // siamese_decoder_add_original: `row` holds the framed original; ownership passes to the
    // decoder on success only (on DuplicateData the caller keeps it), and never when `borrowed`.
    Result add_original(uint32_t packet_num, RowId row, uint32_t framed_bytes, uint32_t header_bytes,
                        uint32_t payload_bytes, void* host, bool* took_ownership, bool borrowed = false);
    // siamese_decoder_add_recovery: `row` holds the packet (data || footer), `tail` the last
    // min(total, 8) bytes of the packet (footer parsing), `host` the whole packet if available.
    // Ownership of `row` passes to the decoder when *took_ownership is set.
    Result add_recovery(RowId row, uint32_t total_bytes, const uint8_t* tail, const uint8_t* host,
                        bool* took_ownership);
    // Batched in-order add_original of columns col0 .. col0 + k - 1 (equal lengths, rows[0..k))
    // while no recovery packet is pending, when is_ready() cannot succeed after any of them.
    // Returns false, with nothing done, when that does not hold.
    bool add_run_inorder(uint32_t col0, const RowId* rows, uint32_t k, uint32_t framed_bytes,
                         uint32_t header_bytes, uint32_t payload_bytes, bool borrowed,
                         uint64_t layout = 0);
    Result is_ready();
    // siamese_decode: recovered packets are appended to `out` (increasing packet number).
    Result decode(std::vector<RecoveredPacket*>& out);
    // `recovered_now`: a packet the decode just returned, looked up even when that decode disabled
    // the decoder on its way out (its removal step can, SiameseDecoder.cpp:1778-2033): the reference
    // still hands those packets to the caller (siamese.cpp:257-270, Decoder::Decode).
    Result get(uint32_t packet_num, StoredOriginal** out, bool recovered_now = false);
    Result ack(uint8_t* buffer, uint32_t limit, uint32_t* used);
    void stats(uint64_t* out, unsigned n);

    bool disabled() const { return disabled_; }
    void set_disabled() { disabled_ = true; }

    // Recovered packets of the latest successful decode (for readback by the C-ABI layer).
    std::vector<RecoveredPacket>& recovered() { return recovered_; }
    // After readback: the exact framed length of a recovered original.
    void set_recovered_length(uint32_t packet_num, uint32_t framed_bytes, uint32_t header_bytes, void* host);

    void pre_flush() override;
    void post_flush() override {}

private:
    // Received originals are stored as segments (encoder.h Segment: runs of equally long packets
    // at fixed row strides, added in order); seg[bit] names the element's segment, or kSingle
    // when the element is described by orig[bit] instead -- a recovered original, one delivered
    // out of order into a hole, a C-ABI add with a host copy -- or is not received (bytes 0).
    static const uint32_t kSingle = 0xffffffffu;
    struct Subwindow {
        uint64_t got = 0;
        uint32_t got_count = 0;
        // bits: orig[] slots written with something to release (an owned row or a host copy) since
        // the subwindow was last cleared (the others are cleared by zeroing; empty slot = all zero)
        uint64_t held = 0;
        uint64_t singles = 0;  // bits: orig[] slots written since the last clear (0: nothing to clear)
        uint32_t seg[kSubwindow];
        StoredOriginal orig[kSubwindow];
        Subwindow() { memset(seg, 0xff, sizeof(seg)); }
    };
    struct Recovery {
        Recovery* next = nullptr;
        Recovery* prev = nullptr;
        RecoveryMeta meta;
        uint32_t element_start = 0, element_end = 0, lost_count = 0;
        RowId row = kNoRow;   // the received packet (owned)
        Sym buf;              // Buffer contents (symbolic)
        uint32_t bytes = 0;   // Buffer.Bytes
    };
    // DecoderColumnLane (SiameseDecoder.h:121-137): the reference keeps ElementStart/End per
    // sum, but every path sets them for all three sums of a lane together and reads are
    // monotone in the element, so one range per lane drives the lane's three sums.
    struct LaneSum {
        uint32_t element_start = 0, element_end = 0;
        LaneSums sums;
    };
    struct MatRow { Recovery* rec = nullptr; bool used = false; uint32_t mcols = 0; };
    struct MatCol { StoredOriginal* orig = nullptr; uint32_t column = 0; uint8_t cx = 0; };

    Context* ctx_;
    uint32_t row_bytes_;
    HostRelease release_;
    void* user_;
    uint64_t stats_[11] = {0};
    bool disabled_ = false;

    // ---- DecoderPacketWindow (SiameseDecoder.h:288-419) ----
    uint32_t count_ = 0, column_start_ = 0, next_expected_ = 0;
    std::vector<Subwindow*> subs_;
    Ring<Segment> segs_;      // run segments in element order; segs_[i] is number seg_base_ + i
    uint32_t seg_base_ = 0;
    uint32_t base_ = 0;       // absolute element number of window element 0
    StoredOriginal view_;     // get() of an element inside a segment
    LaneSum lanes_[kLanes];
    uint32_t sum_column_start_ = 0, sum_column_count_ = 0;
    std::vector<RecoveredPacket> recovered_;
    bool has_recovered_ = false;
    std::vector<uint32_t> recovered_columns_;

    // ---- RecoveryPacketList ----
    Recovery* head_ = nullptr;
    Recovery* tail_ = nullptr;
    // list_insert's last insertion (node, its end and column start) and the list generation it
    // left (list_gen_ counts every other change of the list or of its nodes' ends): a packet with
    // the same key goes right in front of that node without the walk (list_insert).
    Recovery* ins_last_ = nullptr;
    uint32_t ins_end_ = 0, ins_start_ = 0;
    uint64_t list_gen_ = 0, ins_gen_ = ~0ull;
    // What remove_elements' walk over the recovery list finds (RemoveElements, :1778-1830), kept
    // for the list generation, window start and count it was taken at; list_insert carries it
    // over an insertion that cannot change the walk's sum target or its participants.
    struct ListWalk {
        bool valid = false;
        uint64_t gen = 0;
        uint32_t column_start = 0, count = 0;
        uint32_t min_start = 0, max_bytes = 0;      // every node's element start / bytes
        bool seen_sum = false;                      // the first sum row (SumCount > Cauchy threshold)
        uint32_t target_start = 0, target_count = 0, target_end = 0;  // (its element end)
        uint32_t min_fse = ~0u;                     // other sum rows' first sum elements
        bool invalid = false;                       // one of those is outside the window
    } walk_;
    void list_walk(ListWalk& w) const;
    // Deleted packets stay readable until the checked region and matrix forget them: the
    // reference frees them into its pool allocator, where stale pointers still read the old
    // fields (RecoveryPacketList::DeletePacketsBefore, SiameseDecoder.cpp:2637-2666).
    std::vector<Recovery*> graveyard_;
    std::vector<Recovery*> pool_;  // recycled Recovery objects (keep their buffers' capacity)
    uint32_t recovery_count_ = 0;
    RecoveryMeta last_meta_;
    uint32_t last_bytes_ = 0;

    // ---- CheckedRegionState ----
    struct Checked {
        uint32_t element_start = 0, next_check_start = 0, recovery_count = 0, lost_count = 0;
        Recovery* first = nullptr;
        Recovery* last = nullptr;
        bool solve_failed = false;
    } cr_;
    // Loss counts decode() has not written yet: `lazy_n_` packets from `lazy_from_` on all face
    // `lazy_lost_` losses (decode's walk past a failed solve, Decoder::decode).  Written before
    // anything reads them (generate_matrix) or the list drops packets; a reset forgets them.
    Recovery* lazy_from_ = nullptr;
    uint32_t lazy_n_ = 0, lazy_lost_ = 0;
    void lazy_write();

    // ---- RecoveryMatrixState ----
    std::vector<MatRow> mrows_;
    std::vector<MatCol> mcols_;
    uint32_t prev_next_check_start_ = 0;
    std::vector<uint8_t> mat_;
    uint32_t mat_rows_ = 0, mat_cols_ = 0, mat_stride_ = 0, mat_alloc_rows_ = 0;
    std::vector<uint32_t> pivots_;
    uint32_t ge_resume_pivot_ = 0;

    uint32_t latest_column_ = 0;
    Sym value_;  // scratch
    // Triangular solve in coefficient space (multiply_lower_triangle / back_substitution):
    // tri_[j * L + k] = coefficient of eliminated row k in row j after the lower triangle,
    // tri_b_[j] = row j's length; a recovered value is a list of groups (row k, clip, coef)
    struct Group { uint32_t k, clip; uint8_t coef; };
    std::vector<uint8_t> tri_, tri_acc_;
    std::vector<uint32_t> tri_b_, tri_clips_, tri_gstart_;
    std::vector<Group> tri_groups_;

    // helpers
    uint32_t to_element(uint32_t column) const { return col_sub(column, column_start_); }
    uint32_t to_column(uint32_t element) const { return col_add(element, column_start_); }
    bool invalid_element(uint32_t e) const { return e >= count_; }
    StoredOriginal& elem(uint32_t e) { return subs_[e / kSubwindow]->orig[e % kSubwindow]; }  // its single slot
    uint32_t seg_id(uint32_t e) const { return subs_[e / kSubwindow]->seg[e % kSubwindow]; }
    bool got(uint32_t e) const { return (subs_[e / kSubwindow]->got >> (e % kSubwindow)) & 1u; }
    // The packet of a received or recovered element: row and framed bytes (false: none).
    bool packet(uint32_t e, RowId& row, uint32_t& bytes) const {
        const Subwindow* s = subs_[e / kSubwindow];
        const uint32_t id = s->seg[e % kSubwindow];
        if (id != kSingle) {
            const Segment& sg = segs_[id - seg_base_];
            row = sg.row(e + base_ - sg.first);
            bytes = sg.bytes;
            return true;
        }
        const StoredOriginal& o = s->orig[e % kSubwindow];
        row = o.row;
        bytes = o.bytes;
        return o.bytes > 0;
    }
    // Append received packets rows[0..k) (equally long, no host copy) as elements e0 .. e0 + k - 1
    // at the window end (beyond every segment), extending the last segment while they continue it.
    void append(uint32_t e0, const RowId* rows, uint32_t k, uint32_t framed_bytes, uint32_t header_bytes,
                uint8_t owned,
                uint64_t layout = 0);
    void release_segment(const Segment& s, uint32_t from, uint32_t n);
    uint32_t next_lane_element(uint32_t element, uint32_t lane) const {
        uint32_t n = element - (element % kLanes) + lane;
        if (n < element) n += kLanes;
        return n;
    }
    uint8_t& mat(uint32_t r, uint32_t c) { return mat_[(size_t)r * mat_stride_ + c]; }

    // window
    bool mark_got(uint32_t column);
    uint32_t range_lost(uint32_t start, uint32_t end);
    uint32_t find_next_lost(uint32_t start);
    uint32_t find_next_got(uint32_t start);
    void iterate_next_expected(uint32_t start);
    bool grow_window(uint32_t end);
    LaneSums& get_lane(uint32_t lane, uint32_t element_end);
    bool start_sums(uint32_t element_start, uint32_t buffer_bytes);
    void reset_sums(uint32_t element_start);
    bool plug_sum_holes(uint32_t element_start);
    void remove_elements();
    void drop_original(StoredOriginal& o);
    void read_original(RowId row, uint32_t len, uint8_t coef, Sym& out) const;

    // recovery list / checked region / matrix
    void list_insert(Recovery* r, bool out_of_order);
    void list_delete_before(uint32_t element);
    void free_recovery(Recovery* r);
    void checked_reset();
    void checked_decrement(uint32_t n);
    void matrix_reset();
    void populate_columns(uint32_t old_cols, uint32_t new_cols);
    void populate_rows(uint32_t old_rows, uint32_t new_rows);
    bool generate_matrix();
    bool matrix_resize(uint32_t rows, uint32_t cols, bool keep);
    void resume_ge(uint32_t old_rows, uint32_t rows);
    bool gaussian_elimination();
    bool pivoted_ge(uint32_t pivot_i);
    bool eliminate_row(uint32_t ge_row, uint32_t rem_row, uint32_t pivot_i, uint32_t column_end, uint8_t val_i);

    // solve
    bool add_single_recovery(RowId row, uint32_t data_bytes, const uint8_t* host,
                             const RecoveryMeta& m, bool* took);
    bool check_recovery_possible();
    Result decode_checked_region();
    bool eliminate_original_data();
    bool eliminate_direct(Recovery* rec, uint32_t sum_elem, Sym& buf);
    struct DirectRun { uint32_t e0, n, off, stride, len, col; RowId row; };  // n 0: a single element
    std::vector<DirectRun> drun_;
    std::vector<uint64_t> dpairs_;
    std::vector<uint32_t> dadj_;
    bool multiply_lower_triangle();
    Result back_substitution();
    Result back_substitution_one();
    bool store_recovered(uint32_t ci, Sym& value, uint32_t bytes, bool& iterate);
    Result finish_solve(bool iterate);
};

} // namespace tamd
