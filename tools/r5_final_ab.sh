#!/bin/bash
# Round-5 profile run (GPU suite, smoke, bench lines, rocprof, PMC), then an A/B of the
# OCC=2 paired-tail start (library variants built with GST_EXTRA_CFLAGS=-DGST_KP_OCC2=...).
ROUND=r5 bash tools/final_check.sh || exit $?
timeout -k 10 900 bash tools/ab_r5.sh 2 gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_kp8.so gibbs_student_t_amd/libgst_kp10.so
