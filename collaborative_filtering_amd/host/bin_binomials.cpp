// binomials -- drop-in for binomials.cpp (quadratic-factor graph-signal filter, SURVEY 8f
// item 4): same files as cheby, same output.
#include "cf_filter_cli.hpp"

int main(int, char**) { return cffilt::run(CF_FILTER_BINOMIAL, "binomials"); }
