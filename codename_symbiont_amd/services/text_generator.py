"""text_generator_service: word-bigram Markov chain over NATS (services/text_generator_service).

Behaviour kept from the reference (src/main.rs):
* trained at start-up on one fixed corpus (:170, configurable via SYMB_MARKOV_CORPUS);
* on ``tasks.generation.text`` (GenerateTextTask) generate at most ``max_length`` words -- the
  prompt is logged and ignored (:118-123), generation starts at a random starter (only the first
  word of each training text), stops early at a word without successors (:82-108);
* publish ONE GeneratedTextMessage on ``events.text.generated`` (:125-142).
The chain itself is native (csrc/native/text.cpp MarkovModel).
"""
from __future__ import annotations

import asyncio

from ..text import MarkovModel
from ..utils import log as ulog
from ..wire import GeneratedTextMessage, GenerateTextTask, current_timestamp_ms, subjects
from .base import Service


class TextGeneratorService(Service):
    name = "text_generator_service"

    def __init__(self, *a, seed: int = 0, **kw):
        super().__init__(*a, **kw)
        self.model = MarkovModel(seed)
        self.log.info("[MARKOV_TRAIN] Training Markov model...")
        if self.model.train(self.cfg.markov_corpus):
            self.log.info("[MARKOV_TRAIN] Training complete. Model has %d states. %d starter words.",
                          self.model.num_states(), len(self.model.starters()))
        else:
            self.log.warning("[MARKOV_TRAIN] Not enough words in text to train (need at least 2).")

    async def setup(self) -> None:
        await self.subscribe_loop(subjects.GENERATE_TEXT, self.handle)

    async def handle(self, msg) -> None:
        try:
            task = GenerateTextTask.from_json(msg.data)
        except ValueError as e:
            self.log.warning("[TASK_DESERIALIZE_FAIL] Failed to deserialize GenerateTextTask: %s", e)
            return
        self.log.info("[TEXT_GEN_HANDLER] Received GenerateTextTask (id: %s), max_length: %d",
                      task.task_id, task.max_length)
        if task.prompt is not None:
            self.log.info("[TEXT_GEN_HANDLER] Prompt: %s", task.prompt)
        text = self.model.generate(max(0, int(task.max_length)))
        out = GeneratedTextMessage(task.task_id, text, current_timestamp_ms())
        await self.publish(subjects.TEXT_GENERATED, out.to_json())
        self.log.info("[NATS_PUB_SUCCESS] Successfully published GeneratedTextMessage (task_id: %s)",
                      task.task_id)


def main() -> None:
    ulog.setup(TextGeneratorService.name, "info")
    asyncio.run(TextGeneratorService().run_forever())


if __name__ == "__main__":
    main()
