#!/bin/bash
# Build an A/B variant of libqpgpu.so with extra -D flags for one kernel source (SRC, default
# qp_lane; the other objects are the in-tree build's) into _ab/<name>/libqpgpu.so; register /
# scratch figures of that source's kernels go to _ab/<name>/regs.txt.
# SRCFILE overrides the source text (e.g. an earlier revision: git show REV:path > file).
#   usage: [SRC=qp_wave] [SRCFILE=path] tools/ab_build.sh NAME -DFLAG=V ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/motion-generation-using-quadratic-programs_amd
OUT=$ROOT/_ab/$NAME
rm -rf "$OUT"; mkdir -p "$OUT/tmp"
make -s -C "$PKG" lib/libqpgpu.so
SRC=${SRC:-qp_lane}
# the in-tree build's per-source scheduler flags (Makefile SCHED_<source>)
SCHED=$(make -s -C "$PKG" --no-print-directory -f Makefile -f - print-sched SRCNAME=$SRC <<'MK'
print-sched:
	@echo $(SCHED_$(SRCNAME))
MK
)
# SCHED_OVERRIDE replaces them ("" = LLVM's default scheduler)
SCHED=${SCHED_OVERRIDE-$SCHED}
# the in-tree build's per-source defines (Makefile DEFS_<source>: qp_lane.o leaves the exact
# p = 0 instantiations to qp_lane_p0.o, so an A/B of C2's kernels builds SRC=qp_lane_p0)
DEFS=$(make -s -C "$PKG" --no-print-directory -f Makefile -f - print-defs SRCNAME=$SRC <<'MK'
print-defs:
	@echo $(DEFS_$(SRCNAME))
MK
)
# the fast lane build is the same source with QPGPU_LANE_FAST (qp_lane_fast.hip) and contraction
XF=""; case "$SRC" in qp_lane_fast|qp_wave_fast) XF="-ffp-contract=fast";; esac
for f in qp_layout qp_lane qp_lane_p0 qp_lane_fast qp_small qp_wave qp_wave_fast qp_panel qp_generic qpgpu_api; do [ "$f" = "$SRC" ] || cp "$PKG/lib/$f.o" "$OUT/"; done
(cd "$OUT/tmp" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fPIC \
   -std=c++17 -I"$ROOT/include" -I"$PKG/csrc" $SCHED $DEFS $XF "$@" -c "${SRCFILE:-$PKG/csrc/$SRC.hip}" -o "$OUT/$SRC.o" -save-temps 2>&1 | grep -v warning | grep -v "warnings\? generated" || true)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libqpgpu.so" "$OUT"/*.o
if [ "$SRC" = qp_lane ]; then PAT=qp_lane_kernelILi7ELi14ELi1ELb1ELi6; elif [ "$SRC" = qp_lane_p0 ]; then PAT=qp_lane_kernelILi7ELi14ELi1ELb1ELi0; elif [ "$SRC" = qp_lane_fast ]; then PAT=qp_lane_fast_kernelILi7ELi14ELi1ELb1ELi6; else PAT=${SRC}_kernel; fi
python3 "$ROOT/tools/kernel_regs.py" "$OUT/tmp/$SRC-hip-amdgcn-amd-amdhsa-gfx950.s" "$PAT" > "$OUT/regs.txt"
rm -rf "$OUT/tmp"
cat "$OUT/regs.txt"
