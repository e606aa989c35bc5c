#!/bin/bash
# Build production + diagnostic libraries; exit non-zero on any failure.
set -e
cd /root/repo
python -m gibbs_student_t_amd.build --force 2>&1 | grep -E "error|warning: (?!.*deprecated)" || true
python -c "import os,sys; sys.exit(0 if os.path.getmtime('gibbs_student_t_amd/libgst.so') >= max(os.path.getmtime(f) for f in ['gibbs_student_t_amd/csrc/gst_kernel.hpp','gibbs_student_t_amd/csrc/gst.hip']) else 1)"
python -m gibbs_student_t_amd.build --stamps 2>&1 | grep -E "error" || true
python -c "import os,sys; sys.exit(0 if os.path.getmtime('gibbs_student_t_amd/libgst_stamps.so') >= os.path.getmtime('gibbs_student_t_amd/csrc/gst_kernel.hpp') else 1)"
echo BUILD_OK
