// Error plumbing for the C ABI: every extern "C" entry point runs its body through guarded(),
// which maps exceptions to DDPCA_E* codes and records a thread-local message.
#pragma once
#include <stdexcept>
#include <string>

namespace ddpca {

struct ApiError : std::runtime_error {
    int code;
    ApiError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return 0;
    } catch (const ApiError& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::invalid_argument& e) {
        set_last_error(e.what());
        return -1;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return -1;
    }
}

}  // namespace ddpca
