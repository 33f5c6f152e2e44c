"""TEST INFRASTRUCTURE ONLY — CPU oracle for the PWG generator hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
as the checker / CPU baseline, never as the product path.
"""
