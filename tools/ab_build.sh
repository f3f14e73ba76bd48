#!/bin/bash
# Build the engine of git revision $1 into ab/$2/lib (A/B runs: DYMU_LIBDIR=ab/$2/lib).
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" planning-path_planning_amd include | tar -x -C "$tmp"
make -C "$tmp/planning-path_planning_amd" -j8 >/dev/null
mkdir -p "$root/ab/$name"
rm -rf "$root/ab/$name/lib"
cp -r "$tmp/planning-path_planning_amd/lib" "$root/ab/$name/lib"
rm -rf "$tmp"
echo "built $rev -> ab/$name/lib"
