// cheby -- drop-in for cheby.cpp (Chebyshev graph-signal filter): reads
// coeff* / graph_topology* / graph_signal* from the CWD, writes graph_filtered_signal_1_of_1.
#include "cf_filter_cli.hpp"

int main(int, char**) { return cffilt::run(CF_FILTER_CHEBY, "cheby"); }
