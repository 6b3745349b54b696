#!/usr/bin/env bash
# Drop-in for src/occurrences/run_jellyfish.sh: `run_jellyfish.sh <reads> <k> <sorted_path>`.
# Same contract (run_jellyfish.sh:3-6): write the "<KMER> <count>" dump of canonical k-mers with
# count >= 2 in LC_ALL=C order to <sorted_path>, counted on the GPU by bin/run_jellyfish.
# HGA_BIN names the directory holding run_jellyfish (default: ../bin next to this script).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
BIN="${HGA_BIN:-$HERE/../bin}"
"$BIN/run_jellyfish" "$1" "$2" "$3"
