"""CPU oracle — TEST INFRASTRUCTURE ONLY (checker for tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py).  Nothing in fm_spark_amd imports this package."""
