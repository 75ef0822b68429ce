"""oracle/ — CPU restatements of the reference's path-trace path.

TEST INFRASTRUCTURE ONLY: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package.  The product never does.
"""
