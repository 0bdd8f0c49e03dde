// common.hpp — error plumbing shared by the C-ABI translation units.
#pragma once
#include <string>

namespace rthost {
// Stores a per-thread message for rt_last_error() and returns `code`.
int set_error(int code, const std::string& msg);
void clear_error();
}  // namespace rthost
