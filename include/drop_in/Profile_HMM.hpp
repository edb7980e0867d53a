// Profile_HMM.hpp -- forwarding header with the reference's file name (data_readers/Profile_HMM.hpp), so
// the reference's callers (test_hmm_parsing.cpp:1, MSV_HMM.hpp:4) build unchanged against this library.
// Profile_HMM itself is declared in msv_hmm.hpp (same members, layouts and constructor argument).
#pragma once

#include "msv_hmm.hpp"  // include/ (one directory up): -I include/drop_in -I include
