L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
for v in stamps_head stamps_new; do for m in uniform descend; do echo "== $v $m"; BSG_LIBRARY=$L/libbsg_$v.so timeout -k 10 120 python tools/probe/descent_stamps.py $m 2>&1 | grep -v amdgpu.ids || exit 1; done; done
