// random_fasta -- seeded synthetic FASTA in the format of FASTA_files/random_FASTA_generator.py:1-16
// ("> random i" headers, residues uniform over the 20 amino acids, 70 per line), which is unseeded and
// fixed at 3 x 3500; here the count, a length range and the seed are parameters.
//
//   random_fasta OUT.fsa [n=3] [lmin=3500] [lmax=lmin] [seed=0]
//
// std::mt19937_64(seed): lengths uniform in [lmin, lmax], then the residues of each record.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s OUT.fsa [n=3] [lmin=3500] [lmax=lmin] [seed=0]\n", argv[0]);
        return 2;
    }
    const unsigned long long n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 3;
    const unsigned long long lmin = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 3500;
    const unsigned long long lmax = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : lmin;
    const unsigned long long seed = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 0;
    if (lmax < lmin) {
        std::fprintf(stderr, "lmax < lmin\n");
        return 2;
    }
    std::FILE* f = std::fopen(argv[1], "w");
    if (!f) {
        std::perror(argv[1]);
        return 1;
    }
    static const char kAmino[] = "ACDEFGHIKLMNPQRSTVWY";
    constexpr size_t kPerLine = 70;
    std::mt19937_64 rng(seed);
    std::uniform_int_distribution<unsigned long long> len(lmin, lmax);
    std::uniform_int_distribution<int> aa(0, 19);
    std::string line;
    for (unsigned long long i = 0; i < n; ++i) {
        std::fprintf(f, "> random %llu\n", i);
        const unsigned long long L = len(rng);
        for (unsigned long long k = 0; k < L; k += kPerLine) {
            line.clear();
            for (unsigned long long j = k; j < L && j < k + kPerLine; ++j) line.push_back(kAmino[aa(rng)]);
            line.push_back('\n');
            std::fwrite(line.data(), 1, line.size(), f);
        }
    }
    return std::fclose(f) == 0 ? 0 : 1;
}
