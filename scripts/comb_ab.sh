# grouped sliding-window encode: groups of 4 vs 8 repairs
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for g in 4 8; do
    timeout -k 10 200 python scripts/sw_bench.py --sw-group $g 2>/dev/null | grep '^{' | python -c "import json,sys;d=json.loads(sys.stdin.read());print('group', $g, d['encode_ms'], d['decode_wall_ms'], d['verify_ok'])"
  done
done
