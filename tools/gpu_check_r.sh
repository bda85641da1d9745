set -o pipefail
INF_BLASLT_VERBOSE=1 timeout -k 10 90 python -u tools/blaslt_check.py 2>&1 | grep -v amdgpu.ids
