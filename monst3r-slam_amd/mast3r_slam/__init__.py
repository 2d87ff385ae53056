"""Drop-in `mast3r_slam` package: the reference's module paths (main_monster_slam.py:12-25,
tracker2.py:6-16, global_opt2.py:1-8, frame.py:6) resolved onto the MI355X implementation
in `monst3r_slam_amd`, so the reference's SLAM glue imports these names unchanged:

  mast3r_slam.monst3r_utils   load_* / monst3r_* inference + matching, resize_img, ...
  mast3r_slam.matching        match, match_iterative_proj, prep_for_iter_proj, pixel_to_lin
  mast3r_slam.frame           Frame, create_frame, SharedKeyframes, SharedStates, Mode, ...
  mast3r_slam.global_opt2     FactorGraph
  mast3r_slam.geometry        point_to_ray_dist, constrain_points_to_ray, act_Sim3, ...
  mast3r_slam.nonlinear_optimizer   check_convergence, huber
  mast3r_slam.config          config, load_config, set_global_config
  mast3r_slam.evaluate        save_traj, save_full_traj (+ ate)
  mast3r_slam.retrieval_database    RetrievalDatabase, load_retriever
  mast3r_slam.lietorch_utils  as_SE3

Poses are `monst3r_slam_amd.lie.Sim3` objects where the reference holds lietorch.Sim3 (the
same [..., 8] data); register it as `lietorch` when lietorch is absent.
The native operator module is `mast3r_slam_backends` (the sibling package)."""
