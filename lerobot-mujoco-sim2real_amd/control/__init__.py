from .TrajectoryGenerator import CartesianTrajectoryGenerator  # noqa: F401
