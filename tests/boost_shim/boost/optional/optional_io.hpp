// Tests-only stand-in for Boost.Optional's I/O header, which the image lacks.  The reference's
// tests/netcode/detail/test_invert_matrix.cc includes it (line 1) only so Catch can print an
// optional; this repo's detail::invert returns its own printable result type, so <ostream> is
// all the test needs.  Nothing under netcode/ lives here, and no product code includes it.
#pragma once
#include <ostream>
