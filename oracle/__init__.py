"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the gloo allreduce hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
package.  The product (gloo_amd/) never does.  See oracle/gloo_oracle.c for the
restatement and its reference citations.
"""
from .oracle import *  # noqa: F401,F403
