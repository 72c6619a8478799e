mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_filter_robot.py "tests/test_gpu_roadmap.py::test_robot_roadmap_binding" -v --timeout 200 --timeout-method thread > gpurun_out/r03b_newtests.log 2>&1
