/* Force-included into the reference GridWorld.cc translation unit only (oracle
 * build recipe Makefile.ref).  It is NOT a stand-in for anything missing: it
 * restores the six local declarations that the shipped GridWorld.cc:333 lost
 * (a stray token `p`), exactly as SURVEY.md 8c lists them.  Every standard
 * header the TU uses is included first so that their include guards keep the
 * token definition below from reaching library code. */
#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <ios>
#include <iostream>
#include <map>
#include <random>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>
#include <tgmath.h>
#define p \
    const Range *range = type.view_range; \
    int view_x_offset = type.view_x_offset, view_y_offset = type.view_y_offset; \
    int view_left_top_x, view_left_top_y, view_right_bottom_x, view_right_bottom_y; \
    range->get_range_rela_offset(view_left_top_x, view_left_top_y, view_right_bottom_x, view_right_bottom_y); \
    std::vector<int> channel_trans = make_channel_trans(group, group2channel(0), type.n_channel, n_group);
