"""perception_service: URL -> main-content text -> ``data.raw_text.discovered``
(services/perception_service/src/main.rs).

* subscribe ``tasks.perceive.url`` (PerceiveUrlTask), one task per message (:217-243);
* GET with a 15 s timeout and the reference User-Agent (:89-94); like reqwest, 4xx/5xx bodies are
  NOT errors -- whatever page comes back is parsed;
* extraction = native ``html_extract_text`` (same container + text selector order, :100-170);
* empty text -> warning, nothing published (:29-35); otherwise RawTextMessage with a fresh UUIDv4,
  the task URL and the current timestamp (:47-69).
Fixed: the reference slices ``extracted_text[..200]`` for its log line, which
panics on texts shorter than 200 bytes or on a non-UTF-8 boundary; here logging is char-safe.
"""
from __future__ import annotations

import asyncio

from ..text import extract_html_text
from ..utils import log as ulog
from ..wire import PerceiveUrlTask, RawTextMessage, WireError, current_timestamp_ms, generate_uuid, subjects
from .base import Service


class PerceptionService(Service):
    name = "perception_service"

    def __init__(self, *a, fetch=None, **kw):
        super().__init__(*a, **kw)
        self._fetch_override = fetch
        self._session = None

    async def setup(self) -> None:
        await self.subscribe_loop(subjects.PERCEIVE_URL, self.handle)

    async def fetch(self, url: str) -> str:
        if self._fetch_override is not None:
            return await self._fetch_override(url)
        import aiohttp

        if self._session is None:
            self._session = aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=self.cfg.scrape_timeout_s),
                headers={"User-Agent": self.cfg.user_agent})
        async with self._session.get(url) as resp:
            body = await resp.read()
            charset = resp.charset or "utf-8"
            try:
                return body.decode(charset, errors="replace")
            except LookupError:
                return body.decode("utf-8", errors="replace")

    async def scrape(self, url: str) -> str:
        self.log.info("[SCRAPE_URL_CONTENT] Scraping URL: %s", url)
        html = await self.fetch(url)
        loop = asyncio.get_running_loop()
        text, container = await loop.run_in_executor(None, extract_html_text, html)
        if container:
            self.log.info("[SCRAPE_URL_CONTENT] Found content block with selector: %s", container)
        if not text:
            self.log.warning("[SCRAPE_URL_CONTENT] No meaningful text content extracted from %s", url)
        else:
            self.log.info("[SCRAPE_URL_CONTENT] Extracted text (first 200 chars): %s", text[:200])
        return text

    async def handle(self, nmsg) -> None:
        try:
            task = PerceiveUrlTask.from_json(nmsg.data)
        except WireError as e:
            self.log.warning("[TASK_DESERIALIZE_FAIL] Failed to deserialize PerceiveUrlTask: %s", e)
            return
        self.log.info("[TASK] Processing task for URL: %s", task.url)
        try:
            text = await self.scrape(task.url)
        except Exception as e:
            self.log.error("[SCRAPE_FAIL] Failed to scrape URL %s: %s", task.url, e)
            self.metrics.inc("scrape_errors")
            return
        if not text:
            self.log.warning("[SCRAPE_EMPTY] Scraping URL %s yielded no text. Not publishing.", task.url)
            return
        msg = RawTextMessage(generate_uuid(), task.url, text, current_timestamp_ms())
        await self.publish(subjects.RAW_TEXT_DISCOVERED, msg.to_json())
        self.log.info("[NATS_PUB_SUCCESS] Successfully published RawTextMessage (id: %s)", msg.id)

    async def stop(self) -> None:
        await super().stop()
        if self._session is not None:
            await self._session.close()


def main() -> None:
    ulog.setup(PerceptionService.name, "info")
    asyncio.run(PerceptionService().run_forever())


if __name__ == "__main__":
    main()
