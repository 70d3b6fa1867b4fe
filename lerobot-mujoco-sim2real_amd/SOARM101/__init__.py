from .SOARM101_Env import SOARM101Env, SOARM101VecEnv  # noqa: F401
