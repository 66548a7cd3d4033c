"""ORACLE package -- test infrastructure only (see model_np.py / fitoct_oracle.c headers).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
