#!/bin/bash
# Build libnazhip from a git revision's sources into naz_amd/lib/libnazhip_<name>.so, for
# same-box A/B runs against the working tree (scripts/ab.sh).  Usage: build_rev.sh <rev> <name>
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2
tmp=$(mktemp -d)
git archive "$rev" naz_amd/csrc naz_amd/build.py include | tar -x -C "$tmp"
mkdir -p "$tmp/naz_amd/lib"
touch "$tmp/naz_amd/__init__.py"
(cd "$tmp" && python -c "import sys; sys.path.insert(0,'.'); from naz_amd import build; print(build.build())" >/dev/null)
cp "$tmp/naz_amd/lib/libnazhip.so" "naz_amd/lib/libnazhip_$name.so"
rm -rf "$tmp"
echo "naz_amd/lib/libnazhip_$name.so"
