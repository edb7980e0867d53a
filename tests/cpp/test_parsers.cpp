// test_parsers.cpp -- restatement of the reference parser known-answer tests:
//   data_readers/test_hmm_parsing.cpp:19-37   (100.hmm header and 9 probabilities, 5 ULP)
//   data_readers/test_fasta_parsing.cpp:5-15  (fasta_like_example.fsa records)
// Runs on the CPU (no device needed).  Usage: test_parsers <repo_root>
#include <cmath>
#include <cstdio>
#include <limits>
#include <string>
#include <type_traits>

#include "msv_hmm.hpp"

template <class T>
static bool almost_equal(T x, T y, int ulp = 5) {  // test_hmm_parsing.cpp:9-15
    return std::fabs(x - y) <= std::numeric_limits<T>::epsilon() * std::fabs(x + y) * ulp ||
           std::fabs(x - y) < std::numeric_limits<T>::min();
}
static float neg_ln_to_prob(double d) { return std::exp(-1 * static_cast<float>(d)); }

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::printf("test_parsers failed: %s (line %d)\n", #c, __LINE__); \
            return 1;                                                    \
        }                                                                \
    } while (0)

int main(int argc, char** argv) {
    const std::string root = argc > 1 ? argv[1] : ".";
    auto hmm = Profile_HMM(root + "/data/profile_HMMs/100.hmm");
    CHECK(hmm.model_length == 101);
    CHECK(hmm.name == "Pfam-B_229");
    CHECK(almost_equal(hmm.stats_local_msv_mu, static_cast<float>(-9.5678)));
    CHECK(almost_equal(hmm.stats_local_forward_lambda, static_cast<float>(0.71755)));
    CHECK(almost_equal(hmm.insert_emissions[0][0], neg_ln_to_prob(2.68618)));
    CHECK(almost_equal(hmm.transitions[0][6], neg_ln_to_prob(0.0)));
    CHECK(almost_equal(hmm.match_emissions[1][0], neg_ln_to_prob(2.66211)));
    CHECK(almost_equal(hmm.match_emissions[100][19], neg_ln_to_prob(4.01014)));
    CHECK(almost_equal(hmm.insert_emissions[1][19], neg_ln_to_prob(3.61503)));
    CHECK(almost_equal(hmm.transitions[1][1], neg_ln_to_prob(4.09464)));
    CHECK(almost_equal(hmm.insert_emissions[100][19], neg_ln_to_prob(3.61503)));
    CHECK(almost_equal(hmm.transitions[100][5], neg_ln_to_prob(0.0)));
    CHECK(almost_equal(hmm.transitions[100][6], neg_ln_to_prob(0.0)));

    auto fasta_seq = FASTA_protein_sequences(root + "/data/FASTA_files/fasta_like_example.fsa");
    CHECK((fasta_seq.sequences ==
           Protein_sequences{{"#ACDEFGHIKLMNPQTVWY"},
                             {"#ACDKLMNPQTVWYEFGHI"},
                             {"#EFMNRGHIKLMNPQT"},
                             {"#MKMRFFSSPCGKAAVDPADRCKEVQQIRDQHPSKIPVIIERYKGEKQLPVLDKTKFLVPDHVNMSELVKI"
                              "IRRRLQLNPTQAFFLLVNQHSMVSVSTPIADIYEQEKDEDGFLYMVYASQETFGFIRENE"}}));
    CHECK(fasta_seq.packed.size() == 4);
    CHECK(fasta_seq.packed.offsets.back() == 18 + 18 + 15 + 130);

    bool threw = false;
    try {
        Profile_HMM missing(root + "/data/profile_HMMs/does_not_exist.hmm");
    } catch (const msv_error& e) {
        threw = e.status == MSV_ERR_IO;
    }
    CHECK(threw);
    std::printf("test_parsers passed\n");
    return 0;
}
