"""Model zoo used by benchmarks and examples (GPT-3 family, Llama-2/3, ERNIE/BERT)."""
from .gpt import GPTConfig, GPTModel, GPTForPretraining, GPTPretrainingCriterion, gpt_config, GPT_CONFIGS  # noqa: F401
from .llama import (LlamaConfig, LlamaModel, LlamaForCausalLM, llama_config, LLAMA_CONFIGS)  # noqa: F401
from .ernie import (ErnieConfig, ErnieModel, ErnieForSequenceClassification, ErnieForPretraining,  # noqa: F401
                    ErniePretrainingCriterion, ernie_config, ERNIE_CONFIGS, BertConfig, BertModel,
                    BertForSequenceClassification, BertForPretraining)
