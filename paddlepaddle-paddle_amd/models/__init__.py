"""Model zoo used by benchmarks and examples (GPT-3 family, Llama-2, ERNIE/BERT)."""
from .gpt import GPTConfig, GPTModel, GPTForPretraining, GPTPretrainingCriterion, gpt_config, GPT_CONFIGS  # noqa: F401
