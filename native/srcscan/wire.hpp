// Binary wire form of a ScanResult: what the persistent isolated scan child
// (srcscan serve, dmcp/parsers/isolated.py) returns to the service process
// instead of the JSON document -- the parent decodes it natively and builds
// its Python objects and database rows the same way as an in-process scan
// (pymodule.cpp), no JSON encode / decode on either side.
//
// Little-endian: "SSW2", then the ScanResult fields in declaration order;
// strings are u32 length + bytes, vectors u32 count + elements, flags u8;
// the file records (encoded and decoded in parallel) are a u32 count, one
// u32 byte length per record, then the records.
// The decoder treats its input as untrusted (the child parsed an untrusted
// repository): every length and count is checked against the bytes left.
#pragma once

#include <string>
#include <string_view>

#include "srcscan.hpp"

namespace srcscan {

// slim: without the inputs of the scan's own resolution pass (absolute
// paths, imports, parameter type names), which no consumer of a finished
// result reads -- what `srcscan serve` sends (about half the bytes)
std::string encode_result(const ScanResult& r, bool slim = false);
// false (and ``err``) on malformed input; ``out`` is then unspecified
bool decode_result(std::string_view in, ScanResult& out, std::string& err);

}  // namespace srcscan
