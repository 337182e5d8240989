SKIP_SUITE=1 bash tools/r5_pipe.sh r5_pipe2 && bash tools/ab_box.sh r5_noslp t2omca_amd/lib/ab_base.so t2omca_amd/lib/ab_noslp_agent.so t2omca_amd/lib/ab_noslp_mixer.so
