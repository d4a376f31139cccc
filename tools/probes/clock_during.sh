#!/bin/bash
# The shader clock while a command runs: rocm-smi --showclocks sampled every 0.25 s into <out>, the command run in the
# foreground, the sampler stopped by its own PID afterwards. usage: bash tools/probes/clock_during.sh <out> <cmd...>
OUT=$1; shift
( while true; do echo "t=$(date +%s.%N)"; rocm-smi --showclocks 2>/dev/null | grep -E "sclk|fclk|mclk"; sleep 0.25; done ) > "$OUT" &
SAMPLER=$!
"$@"
RC=$?
kill "$SAMPLER" 2>/dev/null
wait "$SAMPLER" 2>/dev/null
exit $RC
