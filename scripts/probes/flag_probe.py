"""Standalone run of tests/test_threads.py::test_device_flag_push_wait_orders_two_streams
with progress prints (a silent exit of the pytest run)."""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
print("start", flush=True)
import test_threads  # noqa: E402

print("imported", flush=True)
test_threads.test_device_flag_push_wait_orders_two_streams()
print("passed", flush=True)
