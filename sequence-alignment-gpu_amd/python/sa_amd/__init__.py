"""Python side of the MI355X sequence-alignment engine.

``sa_amd.engine`` binds the C ABI (include/sa_hip.h); ``sa_amd.synthetic`` makes the benchmark
inputs. Import ``sa_amd.engine`` explicitly: it raises ImportError when the HIP library is not built.
"""
