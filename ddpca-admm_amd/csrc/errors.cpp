#include <string>

#include "../../include/ddpca_amd.h"
#include "common.hpp"

namespace ddpca {
static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace ddpca

extern "C" const char* ddpca_last_error(void) { return ddpca::g_last_error.c_str(); }
