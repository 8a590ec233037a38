"""gsr_amd: host-side support of the MI355X Gaussian rasterizer (libgsr.so).

  _lib       ctypes binding of include/gsr.h (no CPU fallback)
  camera     reference camera maths (getWorld2View2 / getProjectionMatrix / focal2fov)
  synthetic  the seeded synthetic scenes of SURVEY.md 8(d)
  parallel   camera-sharded data parallelism with a bucketed RCCL all-reduce
"""
