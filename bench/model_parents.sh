#!/usr/bin/env bash
# Run the ledger state machine (tests/test_ledger_model.py, as it is in this tree) against the
# parents of round-4 bug fixes, each in its own git worktree, and at HEAD.
#
#   bash bench/model_parents.sh OUT_DIR [COMMIT ...]
#
# For each COMMIT: worktree of COMMIT^ under $TMPDIR, this tree's test file copied in, every
# variant run with GM_MODEL_EXAMPLES x GM_MODEL_STEPS (defaults 25 x 25) and no shrinking.
# OUT_DIR/<commit>.log is pytest's output; OUT_DIR/summary.tsv has one line per commit:
# commit, parent, variants failed, the first finding. Up to $JOBS (default 3) at once.
set -u -o pipefail
OUT=${1:?out dir}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
COMMITS=("$@")
if [ ${#COMMITS[@]} -eq 0 ]; then
    COMMITS=(8f804ea 576377c cb35434 49bf5f0 dd692ae 9cc5468 48de318 e73e592 bebf9a5 868514a
             d3886d3 c862366)
fi
EX=${GM_MODEL_EXAMPLES:-25}
ST=${GM_MODEL_STEPS:-25}
JOBS=${JOBS:-3}
WT=${TMPDIR:-/tmp}/gm-model-parents
mkdir -p "$OUT" "$WT"
OUT=$(cd "$OUT" && pwd)

one() {   # label, worktree rev ("" = this tree)
    local label=$1 rev=$2 dir
    if [ -n "$rev" ]; then
        dir=$WT/$label
        [ -d "$dir" ] || git -C "$ROOT" worktree add -f --detach "$dir" "$rev" > /dev/null 2>&1
        cp "$ROOT/tests/test_ledger_model.py" "$dir/tests/"
    else
        dir=$ROOT
    fi
    (cd "$dir" && GM_MODEL_EXAMPLES=$EX GM_MODEL_STEPS=$ST GM_MODEL_SHRINK=0 \
        timeout 3000 python -m pytest tests/test_ledger_model.py -q -p no:cacheprovider \
        -p no:logging > "$OUT/$label.log" 2>&1)
    local failed finding
    failed=$(grep -oE "^FAILED tests/test_ledger_model.py::[A-Za-z]+" "$OUT/$label.log" \
             | sed 's/.*:://' | tr '\n' ' ')
    finding=$(grep -m1 "^MODEL FINDING" "$OUT/$label.log" | cut -c16-600)
    printf '%s\t%s\t%s\t%s\n' "$label" "${rev:-HEAD}" "${failed:-none}" "${finding:--}" \
        >> "$OUT/summary.tsv"
    echo "$label: failed ${failed:-none}"
}

: > "$OUT/summary.tsv"
one HEAD "" &
for c in "${COMMITS[@]}"; do
    while [ "$(jobs -rp | wc -l)" -ge "$JOBS" ]; do sleep 2; done
    one "$c" "$c^" &
done
wait
for c in "${COMMITS[@]}"; do
    git -C "$ROOT" worktree remove --force "$WT/$c" > /dev/null 2>&1
done
git -C "$ROOT" worktree prune
