export MI355X_DP_S3_ROOT=/tmp/s3 MI355X_DP_JOBS_ROOT=/tmp/jobs
bash tools/gpu_steps.sh \
  nb2_verbatim 900 "python -u tools/run_notebook.py --compat --workdir /tmp/nb2 --report gpurun_out/nb2_verbatim.json ref_fixture/notebooks/2_pytorch_dist_smddp_gpu.ipynb"
bash tools/gpu_steps.sh refprof 700 "bash tools/profile_reference_script.sh 2"
