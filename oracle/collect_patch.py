#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY -- INTEGRATION.md section 2a's call-site changes, applied at build
time to a scratch copy of FPNN's IO plumbing.  No reference text is
committed: this script reads the reference sources where they lie, edits them in memory
and writes the edited copies into the overlay directory oracle/_ref/co/ov/core (git-
ignored), replacing the overlay's symlinks for exactly these four files:

  core/IOBuffer.cpp
    * SendBuffer::encryptData (core/IOBuffer.cpp:36-45): its _encryptor->encrypt(_currBuffer)
      calls become fpnn_io::encrypt(_encryptor, _currBuffer) -- queued in the IO thread's
      EncryptorBatch during a collect phase (oracle/io_collect.h), direct otherwise;
    * SendBuffer::realSend (core/IOBuffer.cpp:47-110) is renamed realSendDirect, unchanged,
      and a new realSend (below) runs in front of it: in a collect phase it dequeues every
      queued frame and hands it to encryptData (so its encryption is queued), keeping the
      frames for the write phase; after the batch's flush the next send() writes those
      frames first, then continues with realSendDirect.
  core/IOBuffer.h       declares realSendDirect and the collected-frame list.
  core/EncryptedPackageReceiver.cpp
    * EncryptedPackageReceiver::fetch (core/EncryptedPackageReceiver.cpp:103-150) is split
      at its "begin decode" comment into fetchStage (take the frame, reset the receiver,
      decrypt through fpnn_io::decrypt -- the call at :110 -- and free the ciphertext
      through fpnn_io::release, deferred past the flush) and fetchDecode (the decode
      and its error handling, as they are); fetch itself becomes fetchStage + fetchDecode,
      so an unchanged caller sees the reference behaviour.  The IO loop calls fetchStage
      for every complete frame, flushes the batch once, then calls fetchDecode.
  core/Receiver.h       declares fetchStage / fetchDecode.

Every anchor is asserted; a reference that moved on fails the build instead of patching
something else.

usage: collect_patch.py <reference root> <overlay root>
"""
import os
import re
import sys


def read(ref, rel):
    with open(os.path.join(ref, rel), encoding="utf-8", errors="surrogateescape") as f:
        return f.read()


def write(ov, rel, text):
    p = os.path.join(ov, rel)
    if os.path.lexists(p):
        os.remove(p)  # the overlay's symlink to the reference file
    with open(p, "w", encoding="utf-8", errors="surrogateescape") as f:
        f.write(text)


def function_span(text, signature):
    """(start, body_open, end) of the function whose definition line matches signature
    (a regex); end is just past its closing brace (braces counted; the reference's bodies
    hold no braces in strings or comments that would unbalance them -- asserted by
    re-parsing the result)."""
    m = re.search(signature, text)
    assert m, f"anchor not found: {signature}"
    i = text.index("{", m.end())
    depth = 0
    for j in range(i, len(text)):
        if text[j] == "{":
            depth += 1
        elif text[j] == "}":
            depth -= 1
            if depth == 0:
                return m.start(), i, j + 1
    raise AssertionError(f"unbalanced body: {signature}")


NEW_REALSEND = r'''

// ---- collect_patch.py (test infrastructure): the cross-connection collector -------------
// A collect phase (fpnn_io::active(), io_collect.h) takes every queued frame and queues
// its encryption in the IO thread's batch through encryptData; the frames are written by
// the next send() after the batch's flush, ahead of anything queued later.
int SendBuffer::realSend(int fd, bool& needWaitSendEvent)
{
	if (fpnn_io::active() && _currBufferProcess == &SendBuffer::encryptData && _currBuffer == NULL)
	{
		std::vector<std::string*> taken;
		{
			std::unique_lock<std::mutex> lck(*_mutex);
			while (_outQueue.size())
			{
				taken.push_back(_outQueue.front());
				_outQueue.pop();
			}
		}
		for (std::string* frame: taken)
		{
			// encryptData's first-package test counts the collected frames ahead of this one
			const uint64_t sentPackage = _sentPackage;
			_sentPackage += _collected.size();
			_currBuffer = frame;
			encryptData();
			_currBuffer = NULL;
			_sentPackage = sentPackage;
			_collected.push_back(frame);
		}
		needWaitSendEvent = false;
		std::unique_lock<std::mutex> lck(*_mutex);
		_sendToken = true;
		return 0;
	}

	uint64_t currSendBytes = 0;
	needWaitSendEvent = false;
	while (!_collected.empty())
	{
		std::string* frame = _collected.front();
		ssize_t n = write(fd, frame->data() + _collectedOffset, frame->length() - _collectedOffset);
		if (n == -1)
		{
			if (errno == EINTR)
				continue;
			const int err = errno;
			std::unique_lock<std::mutex> lck(*_mutex);
			_sentBytes += currSendBytes;
			_sendToken = true;
			if (err == EAGAIN || err == EWOULDBLOCK)
			{
				needWaitSendEvent = true;
				return 0;
			}
			return err;
		}
		_collectedOffset += (size_t)n;
		currSendBytes += (uint64_t)n;
		if (_collectedOffset == frame->length())
		{
			delete frame;
			_collected.pop_front();
			_collectedOffset = 0;
			_sentPackage += 1;
		}
	}
	{
		std::unique_lock<std::mutex> lck(*_mutex);
		_sentBytes += currSendBytes;
	}
	return realSendDirect(fd, needWaitSendEvent);
}
'''


def patch_iobuffer_cpp(t):
    t = '#include <vector>\n#include "io_collect.h"  // collect_patch.py\n' + t
    a, b, e = function_span(t, r"void SendBuffer::encryptData\(\)\s*\n")
    body = t[b:e]
    n = body.count("_encryptor->encrypt(_currBuffer);")
    assert n == 2, f"encryptData: expected 2 encrypt calls, found {n}"
    body = body.replace("_encryptor->encrypt(_currBuffer);", "fpnn_io::encrypt(_encryptor, _currBuffer);")
    t = t[:b] + body + t[e:]
    sig = "int SendBuffer::realSend(int fd, bool& needWaitSendEvent)"
    assert t.count(sig) == 1, "realSend definition"
    t = t.replace(sig, "int SendBuffer::realSendDirect(int fd, bool& needWaitSendEvent)")
    return t + NEW_REALSEND


def patch_iobuffer_h(t):
    decl = "int realSend(int fd, bool& needWaitSendEvent);"
    assert t.count(decl) == 1, "realSend declaration"
    t = t.replace(decl, decl + "\n\t\tint realSendDirect(int fd, bool& needWaitSendEvent);"
                  "\n\t\tstd::deque<std::string*> _collected;\t//-- collect_patch.py: frames awaiting the flush"
                  "\n\t\tsize_t _collectedOffset = 0;", 1)
    t = t.replace("#include <queue>", "#include <queue>\n#include <deque>", 1)
    assert "#include <deque>" in t
    return t


def patch_receiver_h(t):
    c = t.index("class EncryptedPackageReceiver")
    m = re.compile(r"virtual bool fetch\(FPQuestPtr& quest, FPAnswerPtr& answer, bool &isHTTP\);").search(t, c)
    assert m, "EncryptedPackageReceiver::fetch declaration"
    add = ("\n\t\t//-- collect_patch.py: fetch = fetchStage (decrypt, queued in a collect phase) + fetchDecode"
           "\n\t\tbool fetchStage(char*& buf, int& dataLen);"
           "\n\t\tbool fetchDecode(char* buf, int dataLen, FPQuestPtr& quest, FPAnswerPtr& answer, bool &isHTTP);")
    return t[:m.end()] + add + t[m.end():]


def patch_package_receiver_cpp(t):
    a, b, e = function_span(t, r"bool EncryptedPackageReceiver::fetch\(FPQuestPtr& quest, FPAnswerPtr& answer, "
                               r"bool &isHTTP\)\s*\n")
    body = t[b + 1:e - 1]  # between the braces
    mark = body.index("//------- begin decode -------//")
    mark = body.rindex("\n", 0, mark) + 1  # split at the start of the marker's line
    stage, decode = body[:mark], body[mark:]
    for old, new in (("int dataLen = _total;", "dataLen = _total;"),
                     ("char* buf = (char*)malloc(dataLen);", "buf = (char*)malloc(dataLen);"),
                     ("_encryptor.decrypt((uint8_t *)buf, _dataBuffer, dataLen);",
                      "fpnn_io::decrypt(&_encryptor, (uint8_t *)buf, _dataBuffer, dataLen);"),
                     # the queued decrypt reads the ciphertext until the flush
                     ("free(_dataBuffer);", "fpnn_io::release(_dataBuffer);")):
        assert stage.count(old) == 1, f"fetch first half: {old}"
        stage = stage.replace(old, new)
    assert "return rev;" in decode and "free(buf);" in decode
    new = ("bool EncryptedPackageReceiver::fetchStage(char*& buf, int& dataLen)\n{" + stage + "\treturn true;\n}\n\n"
           "bool EncryptedPackageReceiver::fetchDecode(char* buf, int dataLen, FPQuestPtr& quest, "
           "FPAnswerPtr& answer, bool &isHTTP)\n{\n" + decode + "}\n\n"
           "bool EncryptedPackageReceiver::fetch(FPQuestPtr& quest, FPAnswerPtr& answer, bool &isHTTP)\n{\n"
           "\tchar* buf = NULL;\n\tint dataLen = 0;\n\tif (!fetchStage(buf, dataLen))\n\t\treturn false;\n"
           "\treturn fetchDecode(buf, dataLen, quest, answer, isHTTP);\n}")
    t = t[:a] + new + t[e:]
    return '#include "io_collect.h"  // collect_patch.py\n' + t


def main():
    ref, ov = sys.argv[1], sys.argv[2]
    write(ov, "core/IOBuffer.cpp", patch_iobuffer_cpp(read(ref, "core/IOBuffer.cpp")))
    write(ov, "core/IOBuffer.h", patch_iobuffer_h(read(ref, "core/IOBuffer.h")))
    write(ov, "core/Receiver.h", patch_receiver_h(read(ref, "core/Receiver.h")))
    write(ov, "core/EncryptedPackageReceiver.cpp",
          patch_package_receiver_cpp(read(ref, "core/EncryptedPackageReceiver.cpp")))
    print("collect_patch: 4 files patched into", ov)


if __name__ == "__main__":
    main()
