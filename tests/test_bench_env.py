"""bench.py chooses the HIP hardware-queue count inside main(), for its own eager
world-1 runs only: importing it (tests/test_bench_roofline.py does, at collection)
must not change the queue count of the importing process. With 2 queues set at
import, the GPU test process's hipGraph replay of the multi-stream train step
faulted on the host (profiles/r6l_gpu_tests_segv.log)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_importing_bench_leaves_the_hip_queue_count_alone(monkeypatch):
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    sys.modules.pop("bench", None)
    import bench  # noqa: F401
    assert "GPU_MAX_HW_QUEUES" not in os.environ
