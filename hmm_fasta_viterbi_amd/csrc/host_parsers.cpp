// host_parsers.cpp -- HMMER3 profile and FASTA readers of the MSV engine (host side).
//
// Semantics follow the reference parsers; the implementation is our own (whole-file reads,
// one pass, residues packed straight into the device CSR code stream):
//   Profile_HMM               data_readers/Profile_HMM.cpp:8-122
//   FASTA_protein_sequences   data_readers/FASTA_protein_sequences.cpp:9-44
// The float rounding of every parsed value matters for bit-exact scores: probabilities are
// expf(-1 * strtof(token)) exactly as Profile_HMM.cpp:40, with '*' parsing as 0 (p = 1).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <new>
#include <sstream>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include <sys/stat.h>

#include "msv.h"
#include "msv_hmm.hpp"

namespace {

constexpr char kLetters[] = "ACDEFGHIKLMNPQRSTVWY";  // MSV_HMM.cpp:29-31

// 0..19 for the 20 amino acids, 255 for '#' (kept by the reference filter, rejected when
// scored), 254 for any other byte (the record is dropped, FASTA_protein_sequences.cpp:24-41).
struct ResidueLut {
    uint8_t v[256];
    ResidueLut() {
        for (auto& x : v) x = 254;
        for (int i = 0; i < 20; ++i) v[static_cast<unsigned char>(kLetters[i])] = static_cast<uint8_t>(i);
        v[static_cast<unsigned char>('#')] = 255;
    }
};
const ResidueLut kLut;

bool read_file(const char* path, std::string& out) {
    // one fstat-sized fread (the old ifstream -> ostringstream path copied the file twice)
    std::FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    struct stat st {};
    if (fstat(fileno(f), &st) != 0 || !S_ISREG(st.st_mode)) {
        std::fclose(f);
        return false;
    }
    out.resize(static_cast<size_t>(st.st_size));
    const size_t got = out.empty() ? 0 : std::fread(&out[0], 1, out.size(), f);
    std::fclose(f);
    return got == out.size();
}

// Line cursor with std::getline semantics ('\n' separated, '\r' kept).
struct Lines {
    const std::string& s;
    size_t p = 0;
    explicit Lines(const std::string& str) : s(str) {}
    bool next(std::string& line) {
        if (p >= s.size()) return false;
        size_t e = s.find('\n', p);
        if (e == std::string::npos) e = s.size();
        line.assign(s, p, e - p);
        p = e + 1;
        return true;
    }
};

// skip_next_words(view, 1), Profile_HMM.cpp:10-13 (without the npos UB on the last token)
const char* skip_word(const char* c) {
    while (*c && *c != ' ') ++c;
    while (*c == ' ') ++c;
    return c;
}

// read_value_after_tag, Profile_HMM.cpp:15-26: first line whose left-stripped text starts with
// `tag`; returns the text after the first word.
bool value_after_tag(Lines& in, const char* tag, std::string& line, const char*& value) {
    const size_t tl = std::strlen(tag);
    while (in.next(line)) {
        const char* c = line.c_str();
        while (*c == ' ') ++c;
        if (std::strncmp(c, tag, tl) == 0) {
            value = skip_word(c);
            return true;
        }
    }
    return false;
}

template <int N>
Probabilities_array<N> parse_probabilities(const char* c) {  // Profile_HMM.cpp:35-45
    Probabilities_array<N> r{};
    while (*c == ' ') ++c;
    for (int i = 0; i < N; ++i) {
        r[i] = std::exp(-1 * std::strtof(c, nullptr));
        c = skip_word(c);
    }
    return r;
}

msv_status parse_profile(const char* path, Profile_HMM& h) {
    std::string text;
    if (!read_file(path, text)) return MSV_ERR_IO;
    Lines in(text);
    std::string line;
    const char* v = nullptr;

    if (!value_after_tag(in, "NAME", line, v)) return MSV_ERR_PARSE;  // :62-64
    h.name = v;
    if (!value_after_tag(in, "LENG", line, v)) return MSV_ERR_PARSE;  // :66-71
    char* end = nullptr;
    long leng = std::strtol(v, &end, 10);
    if (end == v || leng < 1 || leng > (1 << 20)) return MSV_ERR_PARSE;
    h.model_length = static_cast<size_t>(leng) + 1;  // dummy node M0

    for (int i = 0; i < 3; ++i) {  // :73-94 (STATS LOCAL MSV/VITERBI/FORWARD, any order)
        if (!value_after_tag(in, "STATS", line, v)) return MSV_ERR_PARSE;
        const char* d = skip_word(v);  // skip LOCAL
        const char kind = d[0];
        char* rest = nullptr;
        const char* nums = skip_word(d);
        const float a = std::strtof(nums, &rest);
        const float b = std::strtof(rest, nullptr);
        if (kind == 'M') {
            h.stats_local_msv_mu = a;
            h.stats_local_msv_lambda = b;
        } else if (kind == 'V') {
            h.stats_local_viterbi_mu = a;
            h.stats_local_viterbi_lambda = b;
        } else if (kind == 'F') {
            h.stats_local_forward_theta = a;
            h.stats_local_forward_lambda = b;
        }
    }

    if (!value_after_tag(in, "COMPO", line, v)) return MSV_ERR_PARSE;  // :96-122
    const size_t M = h.model_length;
    h.match_emissions.clear();
    h.insert_emissions.clear();
    h.transitions.clear();
    h.match_emissions.reserve(M);
    h.insert_emissions.reserve(M);
    h.transitions.reserve(M);
    if (!in.next(line)) return MSV_ERR_PARSE;
    h.insert_emissions.push_back(parse_probabilities<NUM_OF_AMINO_ACIDS>(line.c_str()));
    if (!in.next(line)) return MSV_ERR_PARSE;
    h.transitions.push_back(parse_probabilities<NUM_OF_TRANSITIONS>(line.c_str()));
    h.match_emissions.push_back(Probabilities_array<NUM_OF_AMINO_ACIDS>());  // node 0 unused, zero
    char tag[32];
    for (size_t i = 1; i < M; ++i) {
        std::snprintf(tag, sizeof(tag), "%zu", i);
        if (!value_after_tag(in, tag, line, v)) return MSV_ERR_PARSE;
        h.match_emissions.push_back(parse_probabilities<NUM_OF_AMINO_ACIDS>(v));
        if (!in.next(line)) return MSV_ERR_PARSE;
        h.insert_emissions.push_back(parse_probabilities<NUM_OF_AMINO_ACIDS>(line.c_str()));
        if (!in.next(line)) return MSV_ERR_PARSE;
        h.transitions.push_back(parse_probabilities<NUM_OF_TRANSITIONS>(line.c_str()));
    }
    return MSV_OK;
}

struct FastaData {
    std::vector<uint8_t> codes;
    std::vector<uint64_t> offsets{0};
    std::vector<std::string> headers;
    size_t rejected = 0;
};

// One chunk of a FASTA text: [begin, end) starts at a line start; every chunk but the first starts
// with a '>' line, so no record spans two chunks.  codes are written into `out` (pre-sized to the
// chunk length, an upper bound), offsets are chunk-relative record ends.
struct FastaChunk {
    std::vector<uint8_t> codes;
    size_t ncodes = 0;
    std::vector<uint64_t> ends;
    std::vector<std::string> headers;
    size_t rejected = 0;
    msv_status status = MSV_OK;
};

// FASTA_protein_sequences.cpp:9-44: a '>' line opens a record, every other line is appended;
// a record with any symbol outside {'#', 20 amino acids} is dropped (lowercase, 'X', '*', '\r',
// ' ' all reject); empty records are kept.  A non-empty line before the first header is
// undefined behaviour in the reference (sequences.back() on an empty vector, :22); here it is
// MSV_ERR_PARSE, and empty lines before the first header are skipped.
void parse_fasta_chunk(const char* text, size_t begin, size_t end, FastaChunk& c) {
    c.codes.resize(end - begin);
    uint8_t* const out = c.codes.data();
    size_t w = 0, rec_start = 0;
    bool open = false, bad = false;
    size_t p = begin;
    while (p < end) {
        const void* nl = std::memchr(text + p, '\n', end - p);
        const size_t e = nl ? static_cast<size_t>(static_cast<const char*>(nl) - text) : end;
        if (text[p] == '>' && e > p) {
            if (open) {
                if (bad) {
                    w = rec_start;
                    c.headers.pop_back();
                    ++c.rejected;
                } else {
                    c.ends.push_back(w);
                }
            }
            c.headers.emplace_back(text + p + 1, e - p - 1);
            open = true;
            bad = false;
            rec_start = w;
        } else if (!open) {
            if (e > p) {
                c.status = MSV_ERR_PARSE;
                return;
            }
        } else if (!bad) {
            // translate the whole line, then test it: no per-byte branch
            uint8_t any_bad = 0;
            for (size_t k = p; k < e; ++k) {
                const uint8_t v = kLut.v[static_cast<unsigned char>(text[k])];
                out[w + (k - p)] = v;
                any_bad |= static_cast<uint8_t>(v == 254);
            }
            if (any_bad) {
                bad = true;
            } else {
                w += e - p;
            }
        }
        p = e + 1;
    }
    if (open) {
        if (bad) {
            w = rec_start;
            c.headers.pop_back();
            ++c.rejected;
        } else {
            c.ends.push_back(w);
        }
    }
    c.ncodes = w;
}

// Whole-file read, then the text is cut into chunks at '>' line starts and parsed on up to 16 host
// threads (~4 MiB minimum per chunk); chunk results are concatenated in order.
msv_status parse_fasta(const char* path, FastaData& out) {
    std::string text;
    if (!read_file(path, text)) return MSV_ERR_IO;
    const size_t n = text.size();
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const size_t want = std::max<size_t>(1, std::min<size_t>(hw, n / (4u << 20)));
    std::vector<size_t> cut{0};
    for (size_t k = 1; k < want; ++k) {
        size_t q = std::max(cut.back() + 1, n * k / want);
        // next line start that opens a record: "\n>"
        while (q < n) {
            const void* nl = std::memchr(text.data() + q, '\n', n - q);
            if (!nl) {
                q = n;
                break;
            }
            q = static_cast<size_t>(static_cast<const char*>(nl) - text.data()) + 1;
            if (q < n && text[q] == '>') break;
        }
        if (q >= n) break;
        cut.push_back(q);
    }
    cut.push_back(n);
    const size_t nchunks = cut.size() - 1;
    std::vector<FastaChunk> chunks(nchunks);
    {
        std::vector<std::thread> pool;
        for (size_t k = 1; k < nchunks; ++k)
            pool.emplace_back([&, k] { parse_fasta_chunk(text.data(), cut[k], cut[k + 1], chunks[k]); });
        parse_fasta_chunk(text.data(), cut[0], cut[1], chunks[0]);
        for (auto& t : pool) t.join();
    }
    size_t total = 0, records = 0;
    for (const auto& c : chunks) {
        if (c.status != MSV_OK) return c.status;
        total += c.ncodes;
        records += c.ends.size();
    }
    out.codes.resize(total);
    out.offsets.assign(1, 0);
    out.offsets.reserve(records + 1);
    out.headers.clear();
    out.headers.reserve(records);
    out.rejected = 0;
    std::vector<size_t> base(nchunks, 0);
    for (size_t k = 1; k < nchunks; ++k) base[k] = base[k - 1] + chunks[k - 1].ncodes;
    {
        std::vector<std::thread> pool;
        for (size_t k = 1; k < nchunks; ++k)
            pool.emplace_back([&, k] {
                if (chunks[k].ncodes) std::memcpy(out.codes.data() + base[k], chunks[k].codes.data(), chunks[k].ncodes);
            });
        if (chunks[0].ncodes) std::memcpy(out.codes.data(), chunks[0].codes.data(), chunks[0].ncodes);
        for (auto& t : pool) t.join();
    }
    for (size_t k = 0; k < nchunks; ++k) {
        for (uint64_t e : chunks[k].ends) out.offsets.push_back(base[k] + e);
        for (auto& h : chunks[k].headers) out.headers.push_back(std::move(h));
        out.rejected += chunks[k].rejected;
    }
    return MSV_OK;
}

}  // namespace

// ================================================================================================
// C++ classes
// ================================================================================================
Profile_HMM::Profile_HMM(const std::string& file_path) {
    const msv_status s = parse_profile(file_path.c_str(), *this);
    if (s != MSV_OK) throw msv_error(s, std::string(msv_status_string(s)) + ": " + file_path);
}

Packed_sequences Packed_sequences::pack(const Protein_sequences& seqs) {
    Packed_sequences p;
    size_t total = 0;
    for (const auto& s : seqs) total += s.empty() ? 0 : s.size() - 1;
    p.codes.reserve(total);
    p.offsets.reserve(seqs.size() + 1);
    for (const auto& s : seqs) {
        for (size_t i = 1; i < s.size(); ++i) {  // skip the '#' sentinel, MSV_HMM.cpp:100
            const uint8_t c = kLut.v[static_cast<unsigned char>(s[i])];
            if (c >= 20) throw std::out_of_range("residue outside the 20 amino acids");  // MSV_HMM.cpp:101
            p.codes.push_back(c);
        }
        p.offsets.push_back(p.codes.size());
    }
    return p;
}

FASTA_protein_sequences::FASTA_protein_sequences(const std::string& file_path) {
    FastaData d;
    const msv_status s = parse_fasta(file_path.c_str(), d);
    if (s != MSV_OK) throw msv_error(s, std::string(msv_status_string(s)) + ": " + file_path);
    const size_t n = d.offsets.size() - 1;
    sequences.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        std::string q = "#";
        q.reserve(d.offsets[i + 1] - d.offsets[i] + 1);
        for (uint64_t k = d.offsets[i]; k < d.offsets[i + 1]; ++k) q += d.codes[k] < 20 ? kLetters[d.codes[k]] : '#';
        sequences.push_back(std::move(q));
    }
    packed.codes = std::move(d.codes);
    packed.offsets = std::move(d.offsets);
    headers = std::move(d.headers);
    rejected = d.rejected;
}

// ================================================================================================
// C-ABI: parsers
// ================================================================================================
struct msv_hmm {
    Profile_HMM hmm;
    std::vector<float> match, insert, trans;  // flattened views
    explicit msv_hmm(const char* path) : hmm(path) {
        const size_t M = hmm.model_length;
        match.resize(M * 20);
        insert.resize(M * 20);
        trans.resize(M * 7);
        for (size_t i = 0; i < M; ++i) {
            for (int j = 0; j < 20; ++j) {
                match[i * 20 + j] = hmm.match_emissions[i][j];
                insert[i * 20 + j] = hmm.insert_emissions[i][j];
            }
            for (int j = 0; j < 7; ++j) trans[i * 7 + j] = hmm.transitions[i][j];
        }
    }
};

struct msv_fasta {
    FastaData d;
};

extern "C" {

msv_status msv_hmm_read(const char* path, msv_hmm** out) {
    if (!path || !out) return MSV_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    try {
        *out = new msv_hmm(path);
        return MSV_OK;
    } catch (const msv_error& e) {
        return e.status;
    } catch (const std::bad_alloc&) {
        return MSV_ERR_OUT_OF_MEMORY;
    } catch (...) {
        return MSV_ERR_PARSE;
    }
}

void msv_hmm_destroy(msv_hmm* hmm) { delete hmm; }
size_t msv_hmm_model_length(const msv_hmm* hmm) { return hmm ? hmm->hmm.model_length : 0; }
const char* msv_hmm_name(const msv_hmm* hmm) { return hmm ? hmm->hmm.name.c_str() : ""; }
void msv_hmm_stats(const msv_hmm* hmm, float out6[6]) {
    if (!hmm || !out6) return;
    const Profile_HMM& h = hmm->hmm;
    out6[0] = h.stats_local_msv_mu;
    out6[1] = h.stats_local_msv_lambda;
    out6[2] = h.stats_local_viterbi_mu;
    out6[3] = h.stats_local_viterbi_lambda;
    out6[4] = h.stats_local_forward_theta;
    out6[5] = h.stats_local_forward_lambda;
}
const float* msv_hmm_match_emissions(const msv_hmm* hmm) { return hmm ? hmm->match.data() : nullptr; }
const float* msv_hmm_insert_emissions(const msv_hmm* hmm) { return hmm ? hmm->insert.data() : nullptr; }
const float* msv_hmm_transitions(const msv_hmm* hmm) { return hmm ? hmm->trans.data() : nullptr; }

msv_status msv_fasta_read(const char* path, msv_fasta** out) {
    if (!path || !out) return MSV_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    try {
        auto f = std::make_unique<msv_fasta>();
        const msv_status s = parse_fasta(path, f->d);
        if (s != MSV_OK) return s;
        *out = f.release();
        return MSV_OK;
    } catch (const std::bad_alloc&) {
        return MSV_ERR_OUT_OF_MEMORY;
    }
}

void msv_fasta_destroy(msv_fasta* fasta) { delete fasta; }
size_t msv_fasta_count(const msv_fasta* f) { return f ? f->d.offsets.size() - 1 : 0; }
size_t msv_fasta_rejected(const msv_fasta* f) { return f ? f->d.rejected : 0; }
const uint8_t* msv_fasta_codes(const msv_fasta* f) { return f ? f->d.codes.data() : nullptr; }
const uint64_t* msv_fasta_offsets(const msv_fasta* f) { return f ? f->d.offsets.data() : nullptr; }
const char* msv_fasta_header(const msv_fasta* f, size_t i) {
    return (f && i < f->d.headers.size()) ? f->d.headers[i].c_str() : nullptr;
}

msv_status msv_encode_residues(const char* letters, size_t n, uint8_t* codes_out) {
    if ((!letters || !codes_out) && n) return MSV_ERR_INVALID_ARGUMENT;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t c = kLut.v[static_cast<unsigned char>(letters[i])];
        if (c >= 20) return MSV_ERR_BAD_RESIDUE;
        codes_out[i] = c;
    }
    return MSV_OK;
}

}  // extern "C"
