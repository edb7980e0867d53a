// FASTA_protein_sequences.hpp -- forwarding header with the reference's file name
// (data_readers/FASTA_protein_sequences.hpp), so the reference's callers (test_fasta_parsing.cpp:1,
// test_MSV.cpp:1) build unchanged against this library.  The class is declared in msv_hmm.hpp.
#pragma once

#include "msv_hmm.hpp"  // include/ (one directory up): -I include/drop_in -I include
