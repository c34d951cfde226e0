// Host problem object behind ddpca_problem_t: the MCONTACT restatement plus cached views.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "mcontact.hpp"

namespace ddpca {

struct Problem {
    MCONTACT mc;
    bool established = false;
    std::vector<uint8_t> owned;  // subdomains whose operators were built (all after establish())
    std::map<std::string, std::vector<double>> cache_f64;
    std::map<std::string, std::vector<int64_t>> cache_i64;
    std::map<std::string, Csr> cache_csr;
};

}  // namespace ddpca
