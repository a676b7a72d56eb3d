#!/bin/bash
# Build librl.so from the kernel sources of git revision $1 into _lib/variants/librl_$2.so
# (A/B against an earlier head), with build.py's flags and per-source TU flags as they were
# at that revision.
set -e
rev=$1; name=$2
here=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$here" archive "$rev" practice_path_planning_for_formula_student_driverless_amd include | tar -x -C "$tmp"
out="$here/practice_path_planning_for_formula_student_driverless_amd/_lib/variants"
mkdir -p "$out"
python3 - "$tmp" "$out/librl_$name.so" <<'EOF'
import importlib.util, os, sys
tmp, dst = sys.argv[1], sys.argv[2]
spec = importlib.util.spec_from_file_location("rev_build", os.path.join(tmp, "practice_path_planning_for_formula_student_driverless_amd", "build.py"))
B = importlib.util.module_from_spec(spec); spec.loader.exec_module(B)
B._compile_link(B.KERNEL_SRCS, [], dst, os.path.join(tmp, "obj"))
EOF
rm -rf "$tmp"
echo "built $out/librl_$name.so from $rev"
