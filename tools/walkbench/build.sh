#!/bin/bash
# Builds walk_bench (host only: g++ on agent.cpp, linked against the in-tree library for the device
# entry points the walk never calls). PG=1: with -pg for gprof.
set -e
cd "$(dirname "$0")"
R=../..
g++ -O2 -g ${PG:+-pg -fno-ipa-icf} -std=c++17 -pthread -I $R/include -I $R/corrosion_amd/csrc walk_bench.cpp \
    -L $R/corrosion_amd -lcorro_hip -Wl,-rpath,$(cd $R/corrosion_amd && pwd) -L /opt/rocm/lib -Wl,-rpath,/opt/rocm/lib \
    -o walk_bench
