// mums_memhash.hpp -- header-only C++ mirror of libMems' MemHash / MaskedMemHash over the
// C ABI in mums.h (libmums_hip.so).  Same member names, argument meaning and error
// behaviour as the reference (libMems/MemHash.h:38-175, MaskedMemHash.h:25-40,
// MatchFinder.h:46-118): failures throw (the reference throws gnException
// InvalidData / "Gap in genome sequence"; here mums::InvalidData / mums::GapInSequence),
// results come back as a MatchList in the reference's bucket-major order.
//
// This is what a C++ caller links against when it does not have libMems itself; the
// adapter that plugs the same ABI into a real libMems build (HipMemHash : mems::MemHash)
// is shown in INTEGRATION.md.
#pragma once

#include <cstdint>
#include <memory>
#include <ostream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "mums.h"

namespace mums {

struct InvalidData : std::runtime_error { using std::runtime_error::runtime_error; };
struct GapInSequence : std::runtime_error { using std::runtime_error::runtime_error; };

// UngappedLocalAlignment<HybridAbstractMatch<>> reduced to its values (Match.h:26):
// one length and G signed 1-based starts (0 = NO_MATCH, AbstractMatch.h:27).
struct Match {
    uint64_t length = 0;
    std::vector<int64_t> starts;
    int64_t Start(uint32_t seqI) const { return starts[seqI]; }
    uint64_t Length() const { return length; }
    uint32_t SeqCount() const { return (uint32_t)starts.size(); }
    uint32_t Multiplicity() const {
        uint32_t m = 0;
        for (int64_t s : starts) m += s != 0;
        return m;
    }
};

// operator<< of UngappedLocalAlignment (UngappedLocalAlignment.h:200-206)
inline std::ostream& operator<<(std::ostream& os, const Match& m) {
    os << m.length;
    for (int64_t s : m.starts) os << '\t' << s;
    return os;
}

// bmer (SortedMerList.h:43-46): an SML entry, position + its seed mer (GetSeedMer)
struct bmer {
    uint32_t position;
    uint64_t mer;
};

// DNAMemorySML (DNAMemorySML.h:27-51, MemorySML.h:26-54) with SortedMerList construction
// deferred to the GPU.  The reference builds every SML on the CPU before FindMatches
// (MemorySML::Create: FillDnaSeedSML + std::sort, MemorySML.cpp:45-60; called by
// GenericMatchList::CreateMemorySMLs, MatchList.h:409-435, and Aligner.cpp:1181-1184), and
// MemHash's merge then reads them.  Here Create only records the seed pattern and the
// lengths and copies the ASCII into HBM (its own one-genome context); MemHash::FindMatches
// takes the genome from there (mums_genome_device -> mums_add_genome_device) and builds
// keys and the sorted order on the device with everything else.  The few other readers
// (Read / operator[] / FindMer / GetSeedMer: SeedOccurrenceList, FindAll callers) materialise
// the SML on first use from the GPU (mums_build_sml: std::sort(bmer_lessthan) order,
// mums_copy_seed_keys: GetDnaSeedMer) -- no host key or sort work on any path.
class HipSML {
public:
    explicit HipSML(int device = 0) : device_(device) {}
    virtual ~HipSML() { if (ctx_) mums_ctx_destroy(ctx_); }
    HipSML(const HipSML&) = delete;
    HipSML& operator=(const HipSML&) = delete;

    // SortedMerList::Create (SortedMerList.cpp:786-824) + MemorySML::Create (MemorySML.cpp:45-60),
    // the sort deferred: header fields and the sequence only
    virtual void Create(const std::string& seq, uint64_t seed) {
        Clear();
        const uint32_t L = seed ? 64 - __builtin_clzll(seed) - __builtin_ctzll(seed) : 0;
        if (L > 32) throw InvalidData("Mer size is too large");     // SortedMerList.cpp:794-795 (64 / 2 bits)
        if (L == 0) throw InvalidData("Can't have 0 seed length");  // :797-798
        if (!ctx_ && mums_ctx_create(device_, &ctx_) != MUMS_OK)
            throw InvalidData("mums_ctx_create failed (no HIP device?)");
        check(mums_set_seed(ctx_, seed));
        check(mums_add_genome(ctx_, seq.data(), seq.size()));
        seed_ = seed;
        seed_length_ = L;
        length_ = seq.size();
    }
    // MemorySML::Clear (MemorySML.cpp:40-43)
    virtual void Clear() {
        if (ctx_) check(mums_clear(ctx_));
        positions_.clear();
        keys_.clear();
        materialized_ = false;
        seed_ = 0;
        seed_length_ = 0;
        length_ = 0;
    }
    uint64_t Seed() const { return seed_; }                                          // SortedMerList.cpp:251-253
    uint32_t SeedLength() const { return seed_length_; }
    uint32_t SeedWeight() const { return (uint32_t)__builtin_popcountll(seed_); }     // getSeedWeight
    uint64_t Length() const { return length_; }                                      // SortedMerList.cpp:284-286
    // SortedMerList::SMLLength (SortedMerList.cpp:288-295), linear sequences
    uint64_t SMLLength() const { return length_ < seed_length_ ? 0 : length_ - seed_length_ + 1; }
    bool IsCircular() const { return false; }

    // MemorySML::Read (MemorySML.cpp:62-82)
    virtual bool Read(std::vector<bmer>& readVector, uint64_t size, uint64_t offset = 0) {
        materialize();
        readVector.clear();
        if (offset > positions_.size()) return false;
        uint64_t last_mer = offset + size;
        bool success = true;
        if (last_mer > positions_.size()) {
            last_mer = positions_.size();
            success = false;
        }
        for (uint64_t i = offset; i < last_mer; ++i) readVector.push_back(at(i));
        return success;
    }
    // MemorySML::operator[] (MemorySML.cpp:88-94)
    virtual bmer operator[](uint64_t index) {
        materialize();
        if (index >= positions_.size()) throw InvalidData("SML index out of range");
        return at(index);
    }
    // DNAMemorySML::GetSeedMer = SortedMerList::GetDnaSeedMer (SortedMerList.cpp:726-783)
    virtual uint64_t GetSeedMer(uint64_t offset) {
        materialize();
        if (offset >= keys_.size()) throw InvalidData("SML offset out of range");
        return keys_[offset];
    }
    // SortedMerList::FindMer (SortedMerList.cpp:170-179) with bsearch (:380-394)
    virtual bool FindMer(uint64_t query_mer, uint64_t& result) {
        uint64_t last_pos = Length();
        if (last_pos == 0 || last_pos < seed_length_) return false;
        last_pos -= seed_length_;
        result = bsearch(query_mer, 0, last_pos);
        return (*this)[result].mer == query_mer;
    }
    bool Materialized() const { return materialized_; }
    mums_ctx* handle() const { return ctx_; }
    int device() const { return device_; }
    // SMLs materialised by any HipSML of this process (a drop-in FindMatches makes none)
    static uint64_t& Materializations() {
        static uint64_t n = 0;
        return n;
    }

protected:
    void check(int rc) const {
        if (rc == MUMS_OK) return;
        std::string msg = ctx_ ? mums_last_error(ctx_) : "no context";
        if (rc == MUMS_E_GAP) throw GapInSequence(msg);
        throw InvalidData(msg);
    }
    bmer at(uint64_t i) const { return bmer{positions_[i], keys_[positions_[i]]}; }
    uint64_t bsearch(uint64_t q, uint64_t start, uint64_t end) {
        const uint64_t middle = (start + end) / 2;
        const uint64_t mid = (*this)[middle].mer;
        if (mid == q) return middle;
        if (mid < q && middle < end) return bsearch(q, middle + 1, end);
        if (mid > q && start < middle) return bsearch(q, start, middle - 1);
        return middle;   // where it would be if it existed
    }
    void materialize() {
        if (materialized_) return;
        if (!ctx_) throw InvalidData("SML not created");
        const uint64_t m = SMLLength();
        check(mums_find_stage(ctx_, MUMS_STAGE_SEEDS));
        positions_.assign(m, 0);
        keys_.assign(m, 0);
        if (m) {
            check(mums_build_sml(ctx_, 0, positions_.data(), m));
            check(mums_copy_seed_keys(ctx_, 0, keys_.data(), m));
        }
        materialized_ = true;
        ++Materializations();
    }
    int device_ = 0;
    mums_ctx* ctx_ = nullptr;
    uint64_t seed_ = 0, length_ = 0;
    uint32_t seed_length_ = 0;
    bool materialized_ = false;
    std::vector<uint32_t> positions_;   // SML order
    std::vector<uint64_t> keys_;        // GetSeedMer per sequence position
};

struct MatchList : std::vector<Match> {
    std::vector<std::string> seq_table;   // genomes in AddSequence order (MatchList.h:110)
    // the SortedMerList of each sequence (MatchList.h:109); shared by copies of the list
    // as the reference's raw pointers are
    std::vector<std::shared_ptr<HipSML>> sml_table;
    // GenericMatchList::GetDefaultMerSize (MatchList.h:351-357)
    uint32_t GetDefaultMerSize() const {
        uint64_t total = 0;
        for (const auto& s : seq_table) total += s.size();
        return mums_default_seed_weight(seq_table.empty() ? 0 : total / seq_table.size());
    }
    // GenericMatchList::CreateMemorySMLs (MatchList.h:409-435) with deferred SMLs: one
    // HipSML::Create per sequence (no keys, no sort: FindMatches builds them on the device)
    void CreateMemorySMLs(uint32_t mer_size = 0, int seed_rank = 0, int device = 0) {
        if (mer_size == 0) mer_size = GetDefaultMerSize();
        const uint64_t default_seed = (uint64_t)mums_get_seed((int)mer_size, seed_rank);
        sml_table.clear();
        for (const auto& s : seq_table) {
            auto sml = std::make_shared<HipSML>(device);
            sml->Create(s, default_seed);
            sml_table.push_back(std::move(sml));
        }
    }
};

class MemHash {
public:
    explicit MemHash(int device = 0) : device_(device) {
        int rc = mums_ctx_create(device, &ctx_);
        if (rc != MUMS_OK) throw InvalidData("mums_ctx_create failed (no HIP device?)");
    }
    virtual ~MemHash() { if (ctx_) mums_ctx_destroy(ctx_); }
    MemHash(const MemHash&) = delete;
    MemHash& operator=(const MemHash&) = delete;

    // MemHash::Clear / ClearSequences (MemHash.cpp:80-93)
    virtual void Clear() { check(mums_clear(ctx_)); }
    virtual void ClearSequences() { Clear(); }
    // MemHash::SetTableSize (MemHash.cpp:95-102), tolerances (MemHash.h:125-144)
    void SetTableSize(uint32_t n) { table_size_ = n; push_params(); }
    void SetRepeatTolerance(uint32_t t) { repeat_tol_ = t; push_params(); }
    uint32_t GetRepeatTolerance() const { return repeat_tol_; }
    void SetEnumerationTolerance(uint32_t t) { enum_tol_ = t; push_params(); }
    uint32_t GetEnumerationTolerance() const { return enum_tol_; }
    // seed pattern the SMLs are sorted on (SortedMerList::Create; 0 = default weight)
    void SetSeed(uint64_t pattern) { check(mums_set_seed(ctx_, pattern)); }

    // MatchFinder::AddSequence (MatchFinder.cpp:59-87): host ASCII, copied to HBM
    virtual bool AddSequence(const std::string& seq) {
        check(mums_add_genome(ctx_, seq.data(), seq.size()));
        return true;
    }
    // device-resident ASCII (not copied)
    bool AddSequenceDevice(const void* d_ascii, uint64_t n) {
        check(mums_add_genome_device(ctx_, d_ascii, n));
        return true;
    }
    // MatchFinder::AddSequence(SortedMerList*, gnSequence*) (MatchFinder.cpp:59-87): the merge
    // reads the SML's seed pattern; the genome is the deferred SML's device copy (no host copy)
    virtual bool AddSequence(HipSML* sml, const std::string* seq = nullptr) {
        (void)seq;   // the reference keeps it for ExtendMatch only; the device reads the SML's copy
        if (!sml) throw InvalidData("Null SortedMerList pointer");
        if (!sml->handle()) throw InvalidData("SortedMerList not created");
        if (sml->device() != device_) throw InvalidData("SortedMerList lives on another device");
        const void* d = nullptr;
        uint64_t n = 0;
        if (mums_genome_device(sml->handle(), 0, &d, &n) != MUMS_OK) throw InvalidData(mums_last_error(sml->handle()));
        check(mums_set_seed(ctx_, sml->Seed()));
        check(mums_add_genome_device(ctx_, d, n));
        return true;
    }

    // MemHash::FindMatches (MemHash.cpp:109-115): adds ml's sequences -- through its
    // SortedMerLists when it has them (MemHash.cpp:117-127 passes ml.sml_table[i]), else the
    // seq_table ASCII -- finds, fills ml
    virtual void FindMatches(MatchList& ml) {
        add_list(ml);
        check(mums_find(ctx_));
        write_match_log();
        write_progress();
        GetMatchList(ml);
    }
    // MemHash::CreateMatches (MemHash.cpp:104-107)
    virtual bool CreateMatches() {
        check(mums_find(ctx_));
        write_match_log();
        write_progress();
        return true;
    }
    // MemHash::GetMatchList (MemHash.h:182-203): clears the list first
    void GetMatchList(MatchList& ml) const {
        ml.clear();
        uint64_t count = 0;
        uint32_t G = 0;
        check(mums_result_count(ctx_, &count, &G));
        std::vector<uint64_t> len(count);
        std::vector<int64_t> st(count * G);
        if (count) check(mums_result_copy(ctx_, len.data(), st.data()));
        ml.reserve(count);
        for (uint64_t i = 0; i < count; ++i) {
            Match m;
            m.length = len[i];
            m.starts.assign(st.begin() + i * G, st.begin() + (i + 1) * G);
            ml.push_back(std::move(m));
        }
    }
    // MemCount / MemCollisionCount (MemHash.h:94-97)
    uint64_t MemCount() const { return stats().mem_count; }
    uint64_t MemCollisionCount() const { return stats().collision_count; }
    // MemHash::MemTableCount (MemHash.h:100): entries inserted per hash bucket
    void MemTableCount(std::vector<uint32_t>& table_count) const {
        table_count.assign(table_size_, 0);
        check(mums_mem_table_count(ctx_, table_count.data(), table_size_));
    }
    // MemHash::PrintDistribution (MemHash.cpp:253-264): bucket, entries, bases per line
    void PrintDistribution(std::ostream& os) const {
        std::vector<uint32_t> cnt;
        MemTableCount(cnt);
        MatchList ml;
        GetMatchList(ml);
        uint64_t e = 0;
        for (uint32_t i = 0; i < cnt.size(); ++i) {
            uint64_t bases = 0;
            for (uint32_t k = 0; k < cnt[i]; ++k) bases += ml[e++].length;
            os << i << '\t' << cnt[i] << '\t' << bases << '\n';
        }
    }
    // MemHash::WriteFile (MemHash.cpp:301-324): header + every entry, bucket-major
    void WriteFile(std::ostream& os, const std::vector<std::string>& names = {},
                   const std::vector<uint64_t>& lengths = {}) const {
        MatchList ml;
        GetMatchList(ml);
        const size_t G = ml.empty() ? lengths.size() : ml[0].starts.size();
        os << "FormatVersion" << '\t' << 1 << "\n";
        os << "SequenceCount" << '\t' << G << "\n";
        for (size_t g = 0; g < G; ++g) {
            const std::string nm = g < names.size() && !names[g].empty() ? names[g] : "null";
            os << "Sequence" << g << "File" << '\t' << nm << "\n";
            os << "Sequence" << g << "Length" << '\t' << (g < lengths.size() ? lengths[g] : 0) << "\n";
        }
        os << "MatchCount" << '\t' << MemCount() << std::endl;
        for (const Match& m : ml) os << m << "\n";
    }
    // MemHash::FindMatchesFromPosition (MemHash.cpp:117-127)
    virtual void FindMatchesFromPosition(MatchList& ml, const std::vector<uint64_t>& start_points) {
        add_list(ml);
        check(mums_set_start_points(ctx_, start_points.data(), (uint32_t)start_points.size()));
        const int rc = mums_find(ctx_);
        (void)mums_set_start_points(ctx_, nullptr, 0);
        check(rc);
        GetMatchList(ml);
    }
    // MatchFinder::SetOffsetLog (MatchFinder.cpp:152-162): the lines the offset stream
    // received during the last find (start points after every MER_REPEAT_LIMIT restart)
    void WriteOffsetLog(std::ostream& os) const {
        uint64_t rows = 0;
        uint32_t G = 0;
        check(mums_get_offset_log(ctx_, nullptr, 0, &rows, &G));
        std::vector<uint64_t> v(rows * G);
        if (rows) check(mums_get_offset_log(ctx_, v.data(), rows, &rows, &G));
        for (uint64_t r = 0; r < rows; ++r) {
            for (uint32_t g = 0; g < G; ++g) os << (g ? "\t" : "") << v[r * G + g];
            os << std::endl;
        }
    }
    mums_stats stats() const {
        mums_stats s{};
        check(mums_get_stats(ctx_, &s));
        return s;
    }
    mums_ctx* handle() const { return ctx_; }

    // GenericMatchList::MultiplicityFilter / LengthFilter (MatchList.h:636-664), applied on
    // the device copy of the last MatchList before GetMatchList
    void MultiplicityFilter(unsigned mult) { check(mums_multiplicity_filter(ctx_, mult)); }
    void LengthFilter(uint64_t length) { check(mums_length_filter(ctx_, length)); }
    // MemHash::SetMatchLog (MemHash.h:149): every inserted entry of the next FindMatches is
    // written to *log in insertion order (MemHash.cpp:238-241), one `len<TAB>starts` line each
    void SetMatchLog(std::ostream* log) {
        match_log_ = log;
        check(mums_set_match_log(ctx_, log != nullptr));
    }
    // MatchFinder::LogProgress (MatchFinder.cpp:55-56): the merge's progress text ("N%.." per
    // whole percent, MatchFinder.cpp:296-309) is written to *os after every FindMatches
    void LogProgress(std::ostream* os) {
        progress_ = os;
        check(mums_set_progress_log(ctx_, os != nullptr));
    }
    // EliminateOverlaps (Aligner.cpp:62-176) of the last MatchList, on the device
    void EliminateOverlaps() { check(mums_eliminate_overlaps(ctx_)); }
    // a caller's MatchList (M x G starts + lengths) as the current result, e.g. to run
    // EliminateOverlaps / the filters on a list the caller assembled
    void LoadMatches(const std::vector<uint64_t>& lengths, const std::vector<int64_t>& starts, uint32_t G) {
        if (starts.size() != lengths.size() * G) throw InvalidData("starts must be M x G");
        check(mums_load_matches(ctx_, G, lengths.size(), lengths.data(), starts.data()));
    }
    // SeedOccurrenceList::construct + getFrequency (SeedOccurrenceList.h:22-67) for genome g
    std::vector<float> SeedOccurrence(uint32_t genome, uint64_t length) const {
        std::vector<float> f(length);
        check(mums_seed_occurrence(ctx_, genome, f.data(), length));
        return f;
    }

protected:
    void check(int rc) const {
        if (rc == MUMS_OK) return;
        std::string msg = mums_last_error(ctx_);
        if (rc == MUMS_E_GAP) throw GapInSequence(msg);
        throw InvalidData(msg);
    }
    void push_params() { check(mums_set_params(ctx_, repeat_tol_, enum_tol_, table_size_)); }
    void add_list(MatchList& ml) {
        if (ml.sml_table.empty()) {
            for (const auto& s : ml.seq_table) AddSequence(s);
            return;
        }
        if (!ml.seq_table.empty() && ml.seq_table.size() != ml.sml_table.size())
            throw InvalidData("one SortedMerList per sequence required");
        for (size_t i = 0; i < ml.sml_table.size(); ++i)
            AddSequence(ml.sml_table[i].get(), i < ml.seq_table.size() ? &ml.seq_table[i] : nullptr);
    }
    void write_match_log() const {
        if (!match_log_) return;
        uint64_t n = 0;
        uint32_t G = 0;
        uint64_t count = 0;
        check(mums_match_log_copy(ctx_, nullptr, nullptr, 0, &n));
        check(mums_result_count(ctx_, &count, &G));
        std::vector<uint64_t> len(n);
        std::vector<int64_t> st(n * G);
        if (n) check(mums_match_log_copy(ctx_, len.data(), st.data(), n, &n));
        for (uint64_t i = 0; i < n; ++i) {
            (*match_log_) << len[i];
            for (uint32_t g = 0; g < G; ++g) (*match_log_) << '\t' << st[i * G + g];
            (*match_log_) << '\n';
        }
        match_log_->flush();
    }
    void write_progress() const {
        if (!progress_) return;
        uint64_t n = 0;
        check(mums_progress_log_copy(ctx_, nullptr, 0, &n));
        std::string t(n + 1, '\0');
        check(mums_progress_log_copy(ctx_, &t[0], n + 1, &n));
        t.resize(n);
        (*progress_) << t;
        progress_->flush();
    }
    std::ostream* match_log_ = nullptr;
    std::ostream* progress_ = nullptr;
    mums_ctx* ctx_ = nullptr;
    int device_ = 0;
    uint32_t repeat_tol_ = 0, enum_tol_ = 1, table_size_ = 40000;
};

// MaskedMemHash (MaskedMemHash.h:25-40)
class MaskedMemHash : public MemHash {
public:
    explicit MaskedMemHash(int device = 0) : MemHash(device) { check(mums_set_mask(ctx_, 1, 0)); }
    virtual void SetMask(uint64_t seq_mask) { check(mums_set_mask(ctx_, 1, seq_mask)); }
};

// ParallelMemHash (ParallelMemHash.h:29-48): same API, the chunked search of
// ParallelMemHash::FindMatches (ParallelMemHash.cpp:42-121) -- its MatchList, not
// MemHash's, at chunk boundaries.  chunk_size = CHUNK_SIZE (ParallelMemHash.cpp:51).
class ParallelMemHash : public MemHash {
public:
    explicit ParallelMemHash(int device = 0, uint64_t chunk_size = 200000) : MemHash(device) {
        check(mums_set_parallel_compat(ctx_, 1, chunk_size));
    }
};

// PairwiseMatchFinder (PairwiseMatchFinder.h:23-33): MemHash hashing every pair of
// single-copy genomes of a seed group (PairwiseMatchFinder.cpp:37-73).
class PairwiseMatchFinder : public MemHash {
public:
    explicit PairwiseMatchFinder(int device = 0) : MemHash(device) { check(mums_set_pairwise(ctx_, 1)); }
};

// MemHash::FindMatches over several GPUs of this process:
// genome block per device, RCCL communicators from ncclCommInitAll (or the host-staged
// in-process communicator: local = true), one thread per device running mums_shard_run.
// The MatchList is the devices' bucket ranges concatenated = MemHash's bucket-major list.
class ShardedMemHash {
public:
    // slices = false: a contiguous genome block per rank; true: every genome cut into
    // world / G position slices on 64-base bounds (BASELINE config 5: 2 x 3 Gbp over 8 GPUs)
    explicit ShardedMemHash(std::vector<int> devices, bool local = false, bool slices = false)
        : devices_(std::move(devices)), slices_(slices) {
        comms_.assign(devices_.size(), nullptr);
        const int rc = local ? mums_comm_init_local(comms_.data(), (int)devices_.size(), devices_.data())
                             : mums_comm_init_all(comms_.data(), (int)devices_.size(), devices_.data());
        if (rc != MUMS_OK) throw InvalidData("communicator init failed (RCCL)");
    }
    ~ShardedMemHash() {
        ranks_.clear();
        for (mums_comm* c : comms_) mums_comm_destroy(c);
    }
    ShardedMemHash(const ShardedMemHash&) = delete;
    ShardedMemHash& operator=(const ShardedMemHash&) = delete;
    void SetSeed(uint64_t pattern) { seed_ = pattern; }
    void SetTableSize(uint32_t n) { table_size_ = n; }
    // MemHash::SetRepeatTolerance (MemHash.h:125-131) / SetEnumerationTolerance (:137-144) on
    // every rank
    void SetRepeatTolerance(uint32_t t) { repeat_tol_ = t; }
    void SetEnumerationTolerance(uint32_t t) { enum_tol_ = t; }
    // ParallelMemHash's MatchList (ParallelMemHash.cpp:42-121, CHUNK_SIZE = chunk_size): every
    // rank searches a contiguous range of the chunks, the bucket owners re-add the ranks' tables
    // rank after rank (genome blocks only)
    void SetParallelCompat(bool enable, uint64_t chunk_size = 200000) { compat_chunk_ = enable ? chunk_size : 0; }
    // PairwiseMatchFinder's MatchList (PairwiseMatchFinder.cpp:37-73): every rank writes the pair
    // rows of its key range's groups (shard_enum_rows)
    void SetPairwise(bool enable) { pairwise_ = enable; }
    bool AddSequence(const std::string& seq) {
        seqs_.push_back(seq);
        return true;
    }
    // MemHash::FindMatchesFromPosition (MemHash.cpp:117-127): all G start points on every rank
    void FindMatchesFromPosition(MatchList& ml, const std::vector<uint64_t>& start_points) {
        start_points_ = start_points;
        try {
            FindMatches(ml);
        } catch (...) {
            start_points_.clear();
            throw;
        }
        start_points_.clear();
    }
    void FindMatches(MatchList& ml) {
        const size_t W = devices_.size(), G = seqs_.size();
        std::vector<uint64_t> lens(G);
        for (size_t g = 0; g < G; ++g) lens[g] = seqs_[g].size();
        ranks_.clear();
        if (slices_) {   // shard.genome_slices
            if (G == 0 || W % G) throw InvalidData("position slices need a rank count that is a multiple of G");
            uint64_t seed = seed_, total = 0;
            for (uint64_t n : lens) total += n;
            if (!seed) seed = mums_get_seed((int)mums_default_seed_weight(total / G), 0);
            const int L = seed ? 64 - __builtin_clzll(seed) - __builtin_ctzll(seed) : 0;
            const size_t k = W / G;
            for (size_t r = 0; r < W; ++r) {
                const size_t g = r / k, j = r % k;
                const uint64_t m = lens[g] >= (uint64_t)L ? lens[g] - L + 1 : 0;
                auto cut = [&](size_t q) { return q == 0 ? 0 : q == k ? m : (m * q / k) / 64 * 64; };
                const uint64_t b0 = cut(j), b1 = std::max(b0, cut(j + 1));
                auto mh = std::make_unique<MemHash>(devices_[r]);
                mh->SetTableSize(table_size_);
                mh->SetRepeatTolerance(repeat_tol_);
                mh->SetEnumerationTolerance(enum_tol_);
                mh->SetSeed(seed);
                mh->AddSequence(b1 > b0 ? seqs_[g].substr(b0, std::min<uint64_t>(lens[g], b1 + L - 1) - b0) : "");
                if (mums_shard_slice(mh->handle(), (uint32_t)G, lens.data(), (uint32_t)g, b0, b1) != MUMS_OK)
                    throw InvalidData(mums_last_error(mh->handle()));
                ranks_.push_back(std::move(mh));
            }
        }
        size_t g0 = 0;
        for (size_t r = 0; r < (slices_ ? 0 : W); ++r) {   // genome_blocks: earlier ranks take the remainder
            const size_t cnt = G / W + (r < G % W ? 1 : 0);
            auto mh = std::make_unique<MemHash>(devices_[r]);
            mh->SetTableSize(table_size_);
            mh->SetRepeatTolerance(repeat_tol_);
            mh->SetEnumerationTolerance(enum_tol_);
            mh->SetSeed(seed_);
            for (size_t g = g0; g < g0 + cnt; ++g) mh->AddSequence(seqs_[g]);
            if (mums_shard_layout(mh->handle(), (uint32_t)G, (uint32_t)g0, lens.data()) != MUMS_OK)
                throw InvalidData(mums_last_error(mh->handle()));
            ranks_.push_back(std::move(mh));
            g0 += cnt;
        }
        if (compat_chunk_)
            for (auto& mh : ranks_)
                if (mums_set_parallel_compat(mh->handle(), 1, compat_chunk_) != MUMS_OK)
                    throw InvalidData(mums_last_error(mh->handle()));
        if (pairwise_)
            for (auto& mh : ranks_)
                if (mums_set_pairwise(mh->handle(), 1) != MUMS_OK) throw InvalidData(mums_last_error(mh->handle()));
        if (!start_points_.empty())
            for (auto& mh : ranks_)
                if (mums_set_start_points(mh->handle(), start_points_.data(), (uint32_t)start_points_.size()) != MUMS_OK)
                    throw InvalidData(mums_last_error(mh->handle()));
        std::vector<int> rc(W, MUMS_OK);
        std::vector<std::thread> th;
        for (size_t r = 0; r < W; ++r)
            th.emplace_back([&, r] { rc[r] = mums_shard_run(ranks_[r]->handle(), comms_[r], MUMS_STAGE_ALL); });
        for (auto& t : th) t.join();
        for (size_t r = 0; r < W; ++r)
            if (rc[r] != MUMS_OK)
                throw InvalidData(std::string("rank ") + std::to_string(r) + ": " + mums_last_error(ranks_[r]->handle()) +
                                  " " + mums_comm_last_error(comms_[r]));
        ml.clear();
        for (size_t r = 0; r < W; ++r) {
            MatchList part;
            ranks_[r]->GetMatchList(part);
            ml.insert(ml.end(), part.begin(), part.end());
        }
    }
    const MemHash& rank(size_t r) const { return *ranks_[r]; }

private:
    std::vector<int> devices_;
    bool slices_ = false;
    std::vector<mums_comm*> comms_;
    std::vector<std::unique_ptr<MemHash>> ranks_;
    std::vector<std::string> seqs_;
    uint64_t seed_ = 0;
    uint32_t table_size_ = 40000;
    uint32_t repeat_tol_ = 0, enum_tol_ = 1;
    uint64_t compat_chunk_ = 0;   // ParallelMemHash compat: CHUNK_SIZE (0: MemHash)
    bool pairwise_ = false;
    std::vector<uint64_t> start_points_;
};

}  // namespace mums
