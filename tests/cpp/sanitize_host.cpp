// sanitize_host.cpp -- host-only driver for the sanitizer builds (csrc/Makefile `asan`, `tsan`).
//
// Exercises every host translation unit with no GPU: the .hmm parser (all 24 profiles, truncated
// files, a last line without its newline -- the reference's remove_prefix(npos) site,
// Profile_HMM.cpp:10-11), the FASTA reader (the golden edge cases, first-line / EOF cases -- the
// reference's sequences.back() on an empty vector, FASTA_protein_sequences.cpp:22 -- and a file large
// enough for the multi-threaded chunked path), the precompute (MSV_HMM.cpp:35-57) and the CPU DP
// (MSV_HMM.cpp:74-113) against the golden scores, msv_shard_bounds, and the Viterbi stage's table builder
// and CPU DP (msv_hmm_viterbi_scores, msv_vit_cpu_score).
// Usage: sanitize_host <repo_root>
#include <dirent.h>
#include <unistd.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "host_cpu.h"
#include "msv.h"
#include "msv_hmm.hpp"

static int failures = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::printf("sanitize_host: FAILED %s (line %d)\n", #c, __LINE__); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

static std::string slurp(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static void spit(const std::string& path, const std::string& text) {
    std::ofstream f(path, std::ios::binary);
    f << text;
}

struct Table {
    std::vector<float> e;
    size_t M = 0;
    float bmk = 0, ec = 0, ej = 0;
};

static bool load_table(const std::string& path, Table& t) {
    msv_hmm* h = nullptr;
    if (msv_hmm_read(path.c_str(), &h) != MSV_OK) return false;
    t.M = msv_hmm_model_length(h);
    t.e.assign(20 * t.M, 0.f);
    const bool ok = msv_hmm_msv_scores(h, t.e.data(), &t.bmk, &t.ec, &t.ej) == MSV_OK;
    msv_hmm_destroy(h);
    return ok;
}

static float score(const Table& t, const uint8_t* codes, size_t L) {
    return msv_host::run_on_sequence(t.e.data(), t.M, t.bmk, t.ec, t.ej, codes, L);
}

static uint32_t bits(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    return u;
}

// tests/golden/<file>.tsv: profile, seq, length, score (hex), score
static std::map<std::pair<std::string, int>, float> golden(const std::string& path) {
    std::map<std::pair<std::string, int>, float> g;
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream ss(line);
        std::string prof, hex;
        int seq;
        size_t len;
        ss >> prof >> seq >> len >> hex;
        g[{prof, seq}] = static_cast<float>(std::strtod(hex.c_str(), nullptr));
    }
    return g;
}

static void check_scores(const std::string& root, const std::string& fasta, const std::string& gold,
                         const std::vector<std::string>& profiles) {
    msv_fasta* f = nullptr;
    CHECK(msv_fasta_read((root + "/data/FASTA_files/" + fasta).c_str(), &f) == MSV_OK);
    if (!f) return;
    const auto g = golden(root + "/tests/golden/" + gold);
    size_t checked = 0;
    for (const auto& name : profiles) {
        Table t;
        CHECK(load_table(root + "/data/profile_HMMs/" + name, t));
        for (size_t s = 0; s < msv_fasta_count(f); ++s) {
            const uint64_t* o = msv_fasta_offsets(f);
            const float got = score(t, msv_fasta_codes(f) + o[s], o[s + 1] - o[s]);
            const auto it = g.find({name, static_cast<int>(s)});
            CHECK(it != g.end());
            if (it != g.end()) {
                if (bits(got) != bits(it->second))
                    std::printf("  %s seq %zu: %a vs golden %a\n", name.c_str(), s, got, it->second);
                CHECK(bits(got) == bits(it->second));
                ++checked;
            }
        }
    }
    msv_fasta_destroy(f);
    std::printf("  %s: %zu scores bitwise equal to %s\n", fasta.c_str(), checked, gold.c_str());
}

struct Parsed {
    msv_status status;
    std::vector<uint64_t> lengths;
    std::string codes;
    size_t rejected = 0;
};

static Parsed parse_text(const std::string& dir, const std::string& name, const std::string& text) {
    const std::string path = dir + "/" + name;
    spit(path, text);
    Parsed p;
    msv_fasta* f = nullptr;
    p.status = msv_fasta_read(path.c_str(), &f);
    if (p.status == MSV_OK) {
        const uint64_t* o = msv_fasta_offsets(f);
        for (size_t s = 0; s < msv_fasta_count(f); ++s) p.lengths.push_back(o[s + 1] - o[s]);
        p.codes.assign(reinterpret_cast<const char*>(msv_fasta_codes(f)), o[msv_fasta_count(f)]);
        p.rejected = msv_fasta_rejected(f);
        msv_fasta_destroy(f);
    }
    std::remove(path.c_str());
    return p;
}

int main(int argc, char** argv) {
    const std::string root = argc > 1 ? argv[1] : ".";
    char tmpl[] = "/tmp/msv_sanitize_XXXXXX";
    const char* tmp = mkdtemp(tmpl);
    if (!tmp) return 2;
    const std::string dir = tmp;

    // 1. every profile parses; precompute + CPU DP equal the reference's golden scores bit for bit
    std::vector<std::string> profiles;
    if (DIR* d = opendir((root + "/data/profile_HMMs").c_str())) {
        while (dirent* e = readdir(d)) {
            const std::string n = e->d_name;
            if (n.size() > 4 && n.substr(n.size() - 4) == ".hmm") profiles.push_back(n);
        }
        closedir(d);
    }
    CHECK(profiles.size() == 24);
    check_scores(root, "fasta_like_example.fsa", "example_scores.tsv", profiles);
    check_scores(root, "random_FASTA.fsa", "random_fasta_scores.tsv", {"100.hmm", "1400.hmm", "2405.hmm"});
    {
        Table t;
        CHECK(load_table(root + "/data/profile_HMMs/100.hmm", t));
        CHECK(score(t, nullptr, 0) == -std::numeric_limits<float>::infinity());  // empty -> -inf
    }

    // 2. .hmm edge cases: missing, truncated anywhere, last line without its newline, garbage
    {
        msv_hmm* h = nullptr;
        CHECK(msv_hmm_read((root + "/data/profile_HMMs/none.hmm").c_str(), &h) == MSV_ERR_IO);
        const std::string text = slurp(root + "/data/profile_HMMs/100.hmm");
        Table ref;
        CHECK(load_table(root + "/data/profile_HMMs/100.hmm", ref));
        std::mt19937 rng(7);
        int ok_cuts = 0;
        for (int k = 0; k < 64; ++k) {
            const size_t cut = k < 8 ? static_cast<size_t>(k) : rng() % text.size();
            spit(dir + "/cut.hmm", text.substr(0, cut));
            h = nullptr;
            const msv_status s = msv_hmm_read((dir + "/cut.hmm").c_str(), &h);
            CHECK((s == MSV_OK) == (h != nullptr));
            if (h) {
                ++ok_cuts;
                msv_hmm_destroy(h);
            }
        }
        std::printf("  truncated 100.hmm: %d of 64 cuts parsed, the rest refused\n", ok_cuts);
        std::string no_nl = text;
        while (!no_nl.empty() && (no_nl.back() == '\n' || no_nl.back() == '\r')) no_nl.pop_back();
        spit(dir + "/nonl.hmm", no_nl);
        Table t;
        CHECK(load_table(dir + "/nonl.hmm", t));
        CHECK(t.M == ref.M && std::memcmp(t.e.data(), ref.e.data(), t.e.size() * 4) == 0);
        spit(dir + "/garbage.hmm", "HMMER3/f\nNAME x\nLENG abc\n");
        h = nullptr;
        CHECK(msv_hmm_read((dir + "/garbage.hmm").c_str(), &h) != MSV_OK && h == nullptr);
        std::remove((dir + "/cut.hmm").c_str());
        std::remove((dir + "/nonl.hmm").c_str());
        std::remove((dir + "/garbage.hmm").c_str());
    }

    // 3. FASTA: the golden edge cases, then first-line / EOF cases
    {
        Parsed p = parse_text(dir, "edge.fsa", slurp(root + "/tests/golden/edge_cases.fsa"));
        CHECK(p.status == MSV_OK);
        CHECK((p.lengths == std::vector<uint64_t>{20, 0, 5, 12, 10}));
        CHECK(p.rejected == 5);
        CHECK(static_cast<uint8_t>(p.codes[20 + 2]) == 255);  // '#' inside a record: rejected at scoring
        CHECK(parse_text(dir, "empty.fsa", "").status == MSV_OK);
        CHECK(parse_text(dir, "empty.fsa", "").lengths.empty());
        CHECK(parse_text(dir, "nohdr.fsa", "ACDE\n>x\nAC\n").status == MSV_ERR_PARSE);
        p = parse_text(dir, "blank.fsa", "\n\n>x\nAC");
        CHECK(p.status == MSV_OK && (p.lengths == std::vector<uint64_t>{2}));
        p = parse_text(dir, "hdronly.fsa", ">only header");
        CHECK(p.status == MSV_OK && (p.lengths == std::vector<uint64_t>{0}));
        p = parse_text(dir, "gt.fsa", ">a\nAC\n>");
        CHECK(p.status == MSV_OK && p.lengths.size() == 2 && p.lengths[0] == 2);
        msv_fasta* f = nullptr;
        CHECK(msv_fasta_read((dir + "/missing.fsa").c_str(), &f) == MSV_ERR_IO && f == nullptr);
    }

    // 4. a file large enough for the chunked multi-threaded reader (> 4 MiB per chunk), every record
    //    and every rejection known in advance
    {
        static const char kAA[] = "ACDEFGHIKLMNPQRSTVWY";
        std::mt19937_64 rng(11);
        std::string text, want;
        std::vector<uint64_t> lengths;
        size_t rejected = 0;
        while (text.size() < (40u << 20)) {
            const size_t L = rng() % 3000;
            const bool bad = rng() % 17 == 0;
            text += ">r" + std::to_string(lengths.size() + rejected) + "\n";
            std::string seq;
            for (size_t i = 0; i < L; ++i) seq += kAA[rng() % 20];
            if (bad) seq.insert(seq.size() / 2, 1, 'x');
            for (size_t i = 0; i < seq.size(); i += 60) text += seq.substr(i, 60) + "\n";
            if (bad) {
                ++rejected;
            } else {
                lengths.push_back(L);
                for (char c : seq) want += static_cast<char>(std::strchr(kAA, c) - kAA);
            }
        }
        Parsed p = parse_text(dir, "big.fsa", text);
        CHECK(p.status == MSV_OK);
        CHECK(p.lengths == lengths);
        CHECK(p.rejected == rejected);
        CHECK(p.codes == want);
        std::printf("  chunked reader: %zu MiB, %zu records, %zu rejected\n", text.size() >> 20, lengths.size(),
                    rejected);
    }

    // 5. shard bounds: cover, monotone, empty batches and more shards than sequences
    {
        std::vector<uint64_t> off{0, 5, 5, 5, 100, 101, 400};
        for (uint32_t shards : {1u, 2u, 3u, 6u, 8u, 64u}) {
            std::vector<uint64_t> b(shards + 1, 777);
            CHECK(msv_shard_bounds(off.data(), off.size() - 1, shards, b.data()) == MSV_OK);
            CHECK(b[0] == 0 && b[shards] == off.size() - 1);
            for (uint32_t k = 0; k < shards; ++k) CHECK(b[k] <= b[k + 1]);
        }
        std::vector<uint64_t> b(5, 777);
        CHECK(msv_shard_bounds(nullptr, 0, 4, b.data()) == MSV_OK);
        for (uint64_t x : b) CHECK(x == 0);
        CHECK(msv_shard_bounds(off.data(), 6, 0, b.data()) == MSV_ERR_INVALID_ARGUMENT);
    }

    // 7. the Viterbi stage's host side: table builder + CPU DP on every profile, both insert
    // modes, edge lengths; the MSV reduction (m->m = 1, every other transition impossible) equals the MSV DP
    {
        std::mt19937 rng(11);
        for (const std::string& prof : profiles) {
            msv_hmm* h = nullptr;
            CHECK(msv_hmm_read((root + "/data/profile_HMMs/" + prof).c_str(), &h) == MSV_OK);
            if (!h) continue;
            const size_t M = msv_hmm_model_length(h);
            std::vector<float> msc(20 * M), isc(20 * M), tsc(7 * M);
            float b = 0, c = 0, j = 0;
            for (int mode : {0, 1}) {
                CHECK(msv_hmm_viterbi_scores(h, mode, msc.data(), isc.data(), tsc.data(), &b, &c, &j) == MSV_OK);
                for (size_t L : {size_t(0), size_t(1), size_t(2), size_t(65), size_t(300)}) {
                    std::vector<uint8_t> codes(L);
                    for (auto& x : codes) x = static_cast<uint8_t>(rng() % 20);
                    float sc = 0;
                    CHECK(msv_vit_cpu_score(msc.data(), mode ? isc.data() : nullptr, tsc.data(), static_cast<uint32_t>(M),
                                            b, c, j, codes.data(), L, &sc) == MSV_OK);
                    CHECK(L > 0 ? std::isfinite(sc) : sc == -std::numeric_limits<float>::infinity());
                }
            }
            std::vector<float> red(7 * M, -std::numeric_limits<float>::infinity());
            for (size_t k = 0; k < M; ++k) red[k * 7] = 0.0f;
            std::vector<uint8_t> codes(200);
            for (auto& x : codes) x = static_cast<uint8_t>(rng() % 20);
            float v = 0;
            CHECK(msv_vit_cpu_score(msc.data(), nullptr, red.data(), static_cast<uint32_t>(M), b, c, j, codes.data(),
                                    codes.size(), &v) == MSV_OK);
            const float m = msv_host::run_on_sequence(msc.data(), M, b, c, j, codes.data(), codes.size());
            CHECK(std::memcmp(&v, &m, sizeof(float)) == 0);
            const uint8_t bad[3] = {1, 20, 2};
            CHECK(msv_vit_cpu_score(msc.data(), nullptr, tsc.data(), static_cast<uint32_t>(M), b, c, j, bad, 3, &v) ==
                  MSV_ERR_BAD_RESIDUE);
            msv_hmm_destroy(h);
        }
    }

    rmdir(dir.c_str());
    if (failures) {
        std::printf("sanitize_host: %d check(s) failed\n", failures);
        return 1;
    }
    std::printf("sanitize_host passed\n");
    return 0;
}
