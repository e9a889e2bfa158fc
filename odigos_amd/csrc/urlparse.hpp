#pragma once
#include <string>

namespace ose {
// net/url.Parse(raw) -> (.Path, err == nil); see urlparse.cpp
bool go_url_parse_path(const std::string& raw, std::string& path);
}  // namespace ose
