"""Drop-in for src/processing/linepredictor.py: BatchLinePredictor, the client
side of the recognise service (linepredictor.py:11-35)."""
import queue
import time

QGET_WAIT_INTERVAL = 0.1      # common.py args.qget_wait_interval
QGET_WAIT_COUNT = 40000       # common.py args.qget_wait_count


class BatchLinePredictor:
    def __init__(self, server, logger=None):
        self.clientid, self.putq, self.getq = server.register()
        if logger is not None:
            logger.info("receive clientid %s", self.clientid)

    def predict_batch(self, batch_name, img_list, logger=None, wait_interval=QGET_WAIT_INTERVAL,
                      wait_count=QGET_WAIT_COUNT, give_up_after=None):
        """Queue every crop as '<batch_name>_<i>' and collect {i: text}
        (linepredictor.py:17-35). Results of other batches on the queue are
        skipped, as in the reference. Past `wait_count` empty polls it warns
        and keeps waiting like the reference; `give_up_after` (polls) raises
        TimeoutError instead."""
        for i, img in enumerate(img_list):
            self.putq.put((f"{batch_name}_{i}", time.time(), img), block=True)
        if logger is not None:
            logger.debug("put %d imgs to queue put %s", len(img_list), self.clientid)
        pred = {}
        waits = 0
        while len(pred) < len(img_list):
            try:
                imgid, txt = self.getq.get(timeout=wait_interval)
            except queue.Empty:
                waits += 1
                if waits > wait_count and logger is not None:
                    logger.warning("WAITING SERVER TOO LONG ...")
                if give_up_after is not None and waits > give_up_after:
                    raise TimeoutError(f"recognise service returned {len(pred)} of {len(img_list)} lines")
                continue
            batchid, idx = imgid.rsplit("_", 1)
            if batchid != batch_name:
                continue
            pred[int(idx)] = txt
        return pred
