"""RL environment over the device graph. (The reference package also exports its LLM agent and
inference orchestration, src/ah_rag/agent/agent.py / inference.py; those sit outside the MI355X
retrieval core)"""
from .environment import GraphEnvironment
from .gym_env import AHRAGGymEnv

__all__ = ["GraphEnvironment", "AHRAGGymEnv"]
