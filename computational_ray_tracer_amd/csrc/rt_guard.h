// Exception firewall of the C-ABI (include/rtmi355x.h: no C++ exception crosses the boundary).  Every extern "C"
// entry point runs its body inside rtmi::guarded: std::bad_alloc -> RT_E_OOM, any other exception (std::system_error
// from a host thread, ...) -> RT_E_STATE, with the message in rt_last_error when there is a context.  (The reference
// prints and returns an empty optional, Shapes.h:985-989; a library must not terminate its host application.)
#pragma once
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <system_error>

#include "../../include/rtmi355x.h"

namespace rtmi {

// Test hook: RTMI_FAULT_INJECT=bad_alloc | system_error | runtime | other makes every guarded entry point throw that
// exception inside its firewall (tests/test_abi_firewall.py).  Read per call: entry points are not hot.  The release
// entry points (rt_destroy, rt_mesh_free) are exempt: an injected fault there would only leak what they free.
inline void fault_injection_point() {
    const char* f = std::getenv("RTMI_FAULT_INJECT");
    if (!f || !*f) return;
    if (!std::strcmp(f, "bad_alloc")) throw std::bad_alloc();
    if (!std::strcmp(f, "system_error")) throw std::system_error(std::make_error_code(std::errc::resource_unavailable_try_again));
    if (!std::strcmp(f, "runtime")) throw std::runtime_error("injected fault");
    if (!std::strcmp(f, "other")) throw 42;
}

template <class Body, class OnError>
int guarded(Body&& body, OnError&& on_error, bool inject = true) noexcept {
    const char* what = nullptr;
    std::string msg;
    int code = RT_E_STATE;
    try {
        if (inject) fault_injection_point();
        return body();
    } catch (const std::bad_alloc&) {
        code = RT_E_OOM;
        what = "host allocation failed (std::bad_alloc)";
    } catch (const std::system_error& e) {
        what = "system error";
        try { msg = std::string("system error: ") + e.what(); } catch (...) {}
    } catch (const std::exception& e) {
        what = "internal error";
        try { msg = std::string("internal error: ") + e.what(); } catch (...) {}
    } catch (...) {
        what = "unknown internal error";
    }
    try {
        on_error(msg.empty() ? std::string(what) : msg);
    } catch (...) {
    }
    return code;
}

}  // namespace rtmi
