#!/bin/bash
# Disassemble the gfx950 code objects of libskillshot.so into /tmp/isa/*.s and
# print the instruction histogram of one kernel:  tools/isa.sh k_step
set -e
LIB=$(cd "$(dirname "$0")/.." && pwd)/skillshot_learning_amd/lib/libskillshot.so
mkdir -p /tmp/isa && cd /tmp/isa && rm -f libskillshot.so.*
/opt/rocm/lib/llvm/bin/llvm-objdump --offloading "$LIB" >/dev/null 2>&1 || true
mv "$(dirname "$LIB")"/libskillshot.so.[0-9]* /tmp/isa/ 2>/dev/null || true
for f in /tmp/isa/libskillshot.so.*gfx950; do /opt/rocm/lib/llvm/bin/llvm-objdump -d "$f" > "$f.s"; done
K=${1:-k_step}
# (kernels in an anonymous namespace mangle as _ZN12_GLOBAL__N_1<len><name>)
F=$(grep -l "<_Z.*[0-9]${K}[A-Z0-9]" /tmp/isa/libskillshot.so.*.s | head -1)
[ -n "$F" ] || { echo "no kernel $K" >&2; exit 1; }
awk -v k="$K" '/^[0-9a-f]+ <.*>:/{on = ($0 ~ "<_Z.*[0-9]" k "[0-9A-Z]")} on' "$F" > /tmp/isa/$K.s
echo "$K: $(grep -c '^\s' /tmp/isa/$K.s) instructions ($F)"
awk '{print $1}' /tmp/isa/$K.s | grep -v '^$' | sort | uniq -c | sort -rn | head -${2:-25}
