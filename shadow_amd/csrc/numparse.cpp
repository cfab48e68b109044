// numparse.cpp -- the GraphML reader's decimal -> double conversion (graphml.c parse_num).
// std::from_chars is correctly rounded, as strtod is, so the two agree bit for bit on
// every decimal they both accept; it runs several times faster on 17-digit values (a
// C5-sized topology file holds ~6e6 of them).  Anything from_chars does not take the same
// way -- a leading '+', hex floats, overflow / underflow -- goes to strtod.
#include <charconv>
#include <cstdlib>
#include <cstring>
#include <system_error>

// *out = strtod(s, &endp); returns endp != s (something was converted)
extern "C" int gml_strtod(const char* s, double* out) {
    const char* end = s + std::strlen(s);
    double v = 0.0;
    const std::from_chars_result r = std::from_chars(s, end, v);
    if (r.ec == std::errc() && r.ptr != s && *r.ptr != 'x' && *r.ptr != 'X') {
        *out = v;
        return 1;
    }
    char* endp = nullptr;
    *out = std::strtod(s, &endp);
    return endp != s;
}
