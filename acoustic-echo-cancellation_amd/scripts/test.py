"""Stage-2 inference CLI, drop-in for Stage2_lhm/scripts/test.py (same flags,
same output tree); see aec_amd/tester.py.  Multi-GPU:
torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/test.py ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aec_amd.tester import main  # noqa: E402

if __name__ == '__main__':
    main()
