#!/bin/bash
# Builds lib/libngram_search_<name>.so from the library sources of git revision <rev> (the
# baseline arm of an A/B; select it at run time with NGS_LIB=<name>).
# usage (here, repo root): tools/variant_rev.sh <rev> <name>
set -e
REV=$1; NAME=$2
TMP=$(mktemp -d)
git archive "$REV" stringsearchlib_amd/csrc include | tar -x -C "$TMP"
make -s -j8 -C "$TMP/stringsearchlib_amd/csrc" 2>&1 | grep -v "warning\|note:\|^ *[0-9]* |\|^ *|\|~~\|^\s*$" || true
cp "$TMP/stringsearchlib_amd/lib/libngram_search.so" "stringsearchlib_amd/lib/libngram_search_$NAME.so"
rm -rf "$TMP"
echo "built stringsearchlib_amd/lib/libngram_search_$NAME.so from $REV"
